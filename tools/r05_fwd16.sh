#!/bin/bash
# r05: the 16x16x32 forward loop -- GPU parity, in-process A/B against the 32x32x16 loop
# (FWD_HS = 1 / 2), phase stamps of both
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/fwd16; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fwd_hs.py -x -v --timeout 120 --timeout-method thread \
   -p no:cacheprovider > $OUT/pytest.log 2>&1 || exit $?
echo "tests ok" > $OUT/status.txt
for sh in 4,16,2048,64 8,16,4096,128 2,8,4096,64 16,16,2048,64; do
  timeout -k 10 150 python tools/kbench.py --shape $sh --kernel fwd --rounds 7 --iters 20 \
     --variant FWD_HS=1 --variant FWD_HS=2 > $OUT/ab_$sh.log 2>&1 || exit $?
done
timeout -k 10 150 python tools/kbench.py --shape 4,16,2048,64 --kernel step --do ones --rounds 7 --iters 20 \
     --variant FWD_HS=1 --variant FWD_HS=2 > $OUT/ab_step.log 2>&1 || exit $?
echo "ab ok" >> $OUT/status.txt
A=cuda-flash-attention_amd/abl
timeout -k 10 120 python tools/stamps_hs.py --kernel fwd16 --lib $A/fw16_stamps/libfa2amd.so \
  --shape 4,16,2048,64 --shape 8,16,4096,128 > $OUT/stamps16.log 2>&1 || exit $?
echo "stamps ok" >> $OUT/status.txt
