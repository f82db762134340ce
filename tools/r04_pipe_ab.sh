#!/bin/bash
# r04: pipelined dQ loop -- parity, then in-process A/B (DQ_PIPE=0/1) at C3, C5, B2_H8_S4096
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04p; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "dq_pipelined or deterministic" \
   --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || exit $?
echo pytest ok > $OUT/status.txt
for sh in 4,16,2048,64 2,8,4096,64 64,16,2048,64; do
  for d in ones randn; do
    timeout -k 10 200 python tools/kbench.py --shape $sh --kernel dqd --do $d --rounds 9 --iters 20 \
      --variant DQ_PIPE=0,DQ_WAVES=8 --variant DQ_PIPE=1,DQ_WAVES=8 > $OUT/ab_${sh}_$d.log 2>&1 || exit $?
  done
done
echo ab ok >> $OUT/status.txt
