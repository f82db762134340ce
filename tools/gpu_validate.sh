#!/bin/bash
# Round validation, one call: smoke + the whole -m gpu suite, bench line, rocprofv3 kernel
# stats of the same command, PMC passes.  Output: gpurun_out/${TAG:-validate}/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-validate}; mkdir -p $OUT
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
echo "smoke ok" > $OUT/status.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/status.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
echo "bench ok" >> $OUT/status.txt
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py \
    --no-cpu-baseline --no-extras --steps 50 --warmup 20 > $OUT/prof.log 2>&1 || exit $?
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats.csv
echo "prof ok" >> $OUT/status.txt
timeout -k 10 300 bash tools/pmc.sh || exit $?
echo "pmc ok" >> $OUT/status.txt
