#!/bin/bash
# r05: forward row sums over the packed 16-bit P (v_pk_add_f16 partials) -- GPU parity, then
# in-process A/B against abl/fw_vsum (fp32 adds of the unpacked P)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pksum; mkdir -p $OUT
L=cuda-flash-attention_amd
timeout -k 10 500 python -u -m pytest tests/test_gpu_fwd_hs.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v \
   --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || exit $?
echo "tests ok" > $OUT/status.txt
for sh in 4,16,2048,64 2,8,4096,64 8,16,4096,128 1,16,8192,64; do
  timeout -k 10 150 python -u tools/kbench.py --shape $sh --kernel fwd --rounds 9 --iters 20 \
     --lib $L/lib/libfa2amd.so --lib $L/abl/fw_vsum/libfa2amd.so > $OUT/fwd_$sh.log 2>&1 || exit $?
done
echo "ab ok" >> $OUT/status.txt
