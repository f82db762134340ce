#!/bin/bash
# r05: hand-scheduled vs 8-wave dK/dV with the bench's dO = ones (and N(0,1)), kernel and
# whole step, in one process
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/dkhs_ones; mkdir -p $OUT
for sh in 4,16,2048,64 2,8,4096,64 16,16,2048,64; do
  for d in ones randn; do
    timeout -k 10 250 python -u tools/kbench.py --shape $sh --kernel dkdv --kernel step --do $d --rounds 9 --iters 20 \
       --variant DKDV_HS=1 --variant DKDV_HS=0 > $OUT/dk_${sh}_$d.log 2>&1 || exit $?
  done
done
echo "ab ok" > $OUT/status.txt
