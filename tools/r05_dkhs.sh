#!/bin/bash
# r05: hand-scheduled dK/dV schedule variants (cap16, cap16+epg2) against the current
# hand-scheduled loop and the 8-wave default, in one process
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/dkhs; mkdir -p $OUT
L=cuda-flash-attention_amd
A=$L/abl
for sh in 4,16,2048,64 2,8,4096,64 16,16,2048,64 1,16,8192,64; do
  timeout -k 10 250 python -u tools/kbench.py --shape $sh --kernel dkdv --rounds 9 --iters 20 \
     --lib $L/lib/libfa2amd.so --lib $A/dk_c16/libfa2amd.so --lib $A/dk_c16e2/libfa2amd.so \
     --variant DKDV_HS=1 --variant DKDV_HS=0 > $OUT/dk_$sh.log 2>&1 || exit $?
done
echo "ab ok" > $OUT/status.txt
