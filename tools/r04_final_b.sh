#!/bin/bash
# r04 final check, part B: bench line, rocprofv3 kernel stats of the same command, PMC passes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04fb; mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
echo "bench ok" > $OUT/status.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py \
    --no-cpu-baseline --no-extras --steps 50 --warmup 20 > $OUT/prof.log 2>&1 || exit $?
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats.csv
echo "prof ok" >> $OUT/status.txt
timeout -k 10 600 bash tools/pmc.sh || exit $?
echo "pmc ok" >> $OUT/status.txt
