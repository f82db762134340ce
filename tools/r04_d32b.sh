#!/bin/bash
# forward one-round rule at D <= 64: parity of the default plans, then D = 32 default A/Bs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/d32b; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "key_split or shapes_vs_oracle or forward_golden or cli or harness" > $OUT/pytest.log 2>&1 || exit $?
for sh in 2,8,1500,32 2,8,2048,32 1,10,960,32 1,10,960,64; do
  timeout -k 10 150 python tools/kbench.py --shape $sh --kernel fwd --do ones --rounds 9 --variant "" \
    --variant FWD_KS=4,FWD_WAVES=4 --variant FWD_WAVES=4 > $OUT/fwd_$sh.log 2>&1 || exit $?
done
