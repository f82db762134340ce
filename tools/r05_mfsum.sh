#!/bin/bash
# r05 (record; the vsum variant is gone with the row-sum MFMAs): forward row sums on the matrix pipe (ones-row MFMAs) and dK/dV staging loads spread
# over three phases -- GPU parity, then in-process A/Bs against abl/fw_vsum (VALU row sums)
# and abl/dk_nosp (bunched loads; DKDV_HS = 1 both, the 8-wave default beside them)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/mfsum; mkdir -p $OUT
L=cuda-flash-attention_amd
timeout -k 10 500 python -u -m pytest tests/test_gpu_fwd_hs.py tests/test_gpu_bwd_hs.py tests/test_gpu_parity.py -x -v \
   --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || exit $?
echo "tests ok" > $OUT/status.txt
for sh in 4,16,2048,64 2,8,4096,64 8,16,4096,128 1,16,8192,64; do
  timeout -k 10 150 python -u tools/kbench.py --shape $sh --kernel fwd --rounds 7 --iters 20 \
     --lib $L/lib/libfa2amd.so --lib $L/abl/fw_vsum/libfa2amd.so > $OUT/fwd_$sh.log 2>&1 || exit $?
done
for sh in 4,16,2048,64 2,8,4096,64 16,16,2048,64; do
  timeout -k 10 150 python -u tools/kbench.py --shape $sh --kernel dkdv --rounds 7 --iters 20 --variant DKDV_HS=1 \
     --lib $L/lib/libfa2amd.so --lib $L/abl/dk_nosp/libfa2amd.so > $OUT/dk_$sh.log 2>&1 || exit $?
  timeout -k 10 150 python -u tools/kbench.py --shape $sh --kernel dkdv --rounds 7 --iters 20 \
     --variant DKDV_HS=0 --variant DKDV_HS=1 > $OUT/dk0_$sh.log 2>&1 || exit $?
done
echo "ab ok" >> $OUT/status.txt
