#!/bin/bash
# D = 128 small-grid forward / backward plans (wave counts) between the sweep's sizes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/d128; mkdir -p $OUT
for sh in 2,8,512,128 2,8,1024,128 2,8,1500,128 2,8,2048,128; do
  timeout -k 10 150 python tools/kbench.py --shape $sh --kernel fwd --do ones --rounds 7 --variant "" \
    --variant FWD_WAVES=2 --variant FWD_WAVES=4 --variant FWD_WAVES=8 > $OUT/fwd_$sh.log 2>&1 || exit $?
  timeout -k 10 150 python tools/kbench.py --shape $sh --kernel dq --kernel dkdv --do ones --rounds 7 --variant "" \
    --variant DKDV_WAVES=2 --variant DKDV_WAVES=4 > $OUT/bwd_$sh.log 2>&1 || exit $?
done
