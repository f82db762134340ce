#!/bin/bash
# r05: staging loads spread over three phases (fwd, dQ) -- overlap probe,
# GPU parity of the three loops, in-process A/B against the bunched-load builds (abl/*_nosp)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/spread; mkdir -p $OUT
L=cuda-flash-attention_amd
timeout -k 10 120 ./tools/microbench/overlap > $OUT/overlap.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_fwd_hs.py tests/test_gpu_bwd_hs.py -x -v --timeout 120 \
   --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || exit $?
echo "tests ok" > $OUT/status.txt
for sh in 4,16,2048,64 2,8,4096,64 8,16,4096,128; do
  timeout -k 10 150 python -u tools/kbench.py --shape $sh --kernel fwd --rounds 7 --iters 20 \
     --lib $L/lib/libfa2amd.so --lib $L/abl/fw_nosp/libfa2amd.so > $OUT/fwd_$sh.log 2>&1 || exit $?
done
for sh in 4,16,2048,64 2,8,4096,64 16,16,2048,64; do
  timeout -k 10 150 python -u tools/kbench.py --shape $sh --kernel dqd --rounds 7 --iters 20 \
     --lib $L/lib/libfa2amd.so --lib $L/abl/dq_nosp/libfa2amd.so > $OUT/dq_$sh.log 2>&1 || exit $?
done
echo "ab ok" >> $OUT/status.txt
