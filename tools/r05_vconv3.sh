#!/bin/bash
# r05 (record; the vconv3 switch is removed): forward with the V staging convert in P3 instead of P2, in-process A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/vconv3; mkdir -p $OUT
L=cuda-flash-attention_amd
for sh in 8,16,4096,128 4,16,2048,64 2,8,4096,64 1,16,4096,128; do
  timeout -k 10 200 python -u tools/kbench.py --shape $sh --kernel fwd --rounds 9 --iters 20 --lib $L/lib/libfa2amd.so \
     --lib $L/abl/fw_vconv3/libfa2amd.so > $OUT/fwd_$sh.log 2>&1 || exit $?
done
echo "ab ok" > $OUT/status.txt
