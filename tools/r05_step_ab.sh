#!/bin/bash
# r05: the fwd + bwd step (dO = ones, the bench's, and N(0,1)) with the product against
# builds without the packed-P row sums (abl/fw_vsum) and without the spread dQ loads
# (abl/dq_nosp), in one process
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/step_ab; mkdir -p $OUT
L=cuda-flash-attention_amd
A=$L/abl
for sh in 4,16,2048,64 2,8,4096,64 16,16,2048,64; do
  for d in ones randn; do
    timeout -k 10 250 python -u tools/kbench.py --shape $sh --kernel step --do $d --rounds 9 --iters 20 \
       --lib $L/lib/libfa2amd.so --lib $A/fw_vsum/libfa2amd.so --lib $A/dq_nosp/libfa2amd.so > $OUT/step_${sh}_$d.log 2>&1 || exit $?
  done
done
echo "ab ok" > $OUT/status.txt
