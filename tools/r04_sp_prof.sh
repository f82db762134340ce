#!/bin/bash
# r04: kernel-trace breakdown of the single-pass backward at C3 (BWD_SP=1) vs the two-kernel plan
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/spp; mkdir -p $OUT
for v in 0 1; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/p$v -o run --output-format csv -- python3 tools/kbench.py \
     --shape 4,16,2048,64 --kernel bwd --do ones --rounds 3 --iters 20 --variant BWD_SP=$v > $OUT/kb$v.log 2>&1 || exit $?
  f=$(find $OUT/p$v -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/stats_sp$v.csv
done
echo done > $OUT/status.txt
