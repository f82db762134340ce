#!/bin/bash
# r05: the 16x16x32 dQ loop -- GPU parity of the hand-scheduled backward, then in-process
# A/B against the 32x32x16 loop (DQ_HS = 1 / 2), then the diagnostics
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/dq16; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_bwd_hs.py -x -v --timeout 120 --timeout-method thread \
   -p no:cacheprovider > $OUT/pytest.log 2>&1 || exit $?
echo "tests ok" > $OUT/status.txt
for sh in 4,16,2048,64 2,8,4096,64 16,16,2048,64; do
  timeout -k 10 150 python tools/kbench.py --shape $sh --kernel dqd --do randn --rounds 7 --iters 20 \
     --variant DQ_HS=1 --variant DQ_HS=2 > $OUT/ab_$sh.log 2>&1 || exit $?
done
timeout -k 10 150 python tools/kbench.py --shape 4,16,2048,64 --kernel step --do ones --rounds 7 --iters 20 \
     --variant DQ_HS=1 --variant DQ_HS=2 > $OUT/ab_step.log 2>&1 || exit $?
echo "ab ok" >> $OUT/status.txt
bash tools/r05_diag.sh
