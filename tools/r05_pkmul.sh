#!/bin/bash
# r05: hand-scheduled dK/dV with dS = P * dP' on packed fp16 halves (v_pk_mul_f16) -- GPU
# parity, then in-process A/B against abl/dk_pk32 (fp32 products) and the 8-wave default
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pkmul; mkdir -p $OUT
L=cuda-flash-attention_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_bwd_hs.py -x -v --timeout 120 --timeout-method thread \
   -p no:cacheprovider > $OUT/pytest.log 2>&1 || exit $?
echo "tests ok" > $OUT/status.txt
for sh in 4,16,2048,64 2,8,4096,64 16,16,2048,64 1,16,8192,64; do
  timeout -k 10 200 python -u tools/kbench.py --shape $sh --kernel dkdv --rounds 9 --iters 20 \
     --lib $L/lib/libfa2amd.so --lib $L/abl/dk_pk32/libfa2amd.so --variant DKDV_HS=1 --variant DKDV_HS=0 \
     > $OUT/dk_$sh.log 2>&1 || exit $?
done
echo "ab ok" >> $OUT/status.txt
