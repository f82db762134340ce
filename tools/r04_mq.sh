#!/bin/bash
# FWD_MQ=2 forward: parity probe, then in-process A/Bs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/mq; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "query_groups" > $OUT/pytest.log 2>&1 || exit $?
timeout -k 10 150 python tools/r04_mq.py > $OUT/parity.log 2>&1 || exit $?
for sh in 4,16,2048,64 2,8,4096,64 1,16,8192,64 2,8,2048,64; do
  timeout -k 10 150 python tools/kbench.py --shape $sh --kernel fwd --kernel step --do ones --rounds 7 \
    --variant FWD_MQ=1 --variant FWD_MQ=2 > $OUT/ab_$sh.log 2>&1 || exit $?
done
