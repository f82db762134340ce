#!/bin/bash
# r05: the query-split hand-scheduled dK/dV loop -- GPU parity, then in-process A/B against
# the 8-wave 16x16x32 kernel (DKDV_HS = 1 / 0)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/dkdv; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_bwd_hs.py -x -v --timeout 120 --timeout-method thread \
   -p no:cacheprovider > $OUT/pytest.log 2>&1 || exit $?
echo "tests ok" > $OUT/status.txt
for sh in 4,16,2048,64 2,8,4096,64 16,16,2048,64; do
  timeout -k 10 150 python tools/kbench.py --shape $sh --kernel dkdv --do randn --rounds 7 --iters 20 \
     --variant DKDV_HS=0 --variant DKDV_HS=1 > $OUT/ab_$sh.log 2>&1 || exit $?
done
timeout -k 10 150 python tools/kbench.py --shape 4,16,2048,64 --kernel step --do ones --rounds 7 --iters 20 \
     --variant DKDV_HS=0 --variant DKDV_HS=1 > $OUT/ab_step.log 2>&1 || exit $?
echo "ab ok" >> $OUT/status.txt
