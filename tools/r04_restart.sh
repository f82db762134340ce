#!/bin/bash
# r04: forward restart limited to the waves that saw a spike -- spike parity tests, then
# the all-rows worst case and the common case timed again
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/restart; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "restart or rescale or shapes_vs_oracle or forward_golden" \
   --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || exit $?
for sh in 4,16,2048,64 2,8,512,64; do
  for inp in rand spike; do
    timeout -k 10 120 python tools/kbench.py --shape $sh --kernel fwd --inputs $inp --rounds 5 --iters 20 \
      > $OUT/fwd_${sh}_$inp.log 2>&1 || exit $?
  done
done
echo done > $OUT/status.txt
