#!/bin/bash
# r05: the fwd + bwd step with the hand-scheduled forward / dQ (defaults) against the
# compiler-scheduled kernels (FWD_HS = 0, DQ_HS = 0), dO = ones and N(0,1), in one process
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/step_hs; mkdir -p $OUT
for sh in 4,16,2048,64 2,8,4096,64 16,16,2048,64; do
  for d in ones randn; do
    timeout -k 10 250 python -u tools/kbench.py --shape $sh --kernel step --do $d --rounds 9 --iters 20 \
       --variant FWD_HS=-1 --variant FWD_HS=0 --variant DQ_HS=0 --variant FWD_HS=0,DQ_HS=0 > $OUT/step_${sh}_$d.log 2>&1 || exit $?
  done
done
echo "ab ok" > $OUT/status.txt
