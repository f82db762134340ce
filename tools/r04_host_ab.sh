#!/bin/bash
# r04: host-API C5 wall and CPU time, condition-variable D2H thread (this tree) vs the r03
# build's yield spin, alternating libraries three times
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/hostab; mkdir -p $OUT
for i in 1 2 3; do
  for l in lib variants/r03; do
    timeout -k 10 200 python tools/host_api_probe.py --c5-only --shards-on-device0 8 --runs 5 \
      --lib cuda-flash-attention_amd/$l/libfa2amd.so > $OUT/run${i}_$(basename $l).json 2>&1 || exit $?
  done
done
echo done > $OUT/status.txt
