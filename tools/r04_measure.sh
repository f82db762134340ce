#!/bin/bash
# r04: bench line of this tree + rocprofv3 kernel stats + per-kernel clock/power
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04m; mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
echo bench ok > $OUT/status.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extras --steps 50 --warmup 20 > $OUT/prof.log 2>&1 || exit $?
echo prof ok >> $OUT/status.txt
KERNELS="fwd dqd dkdv" timeout -k 10 200 bash tools/clockwatch_kernels.sh || exit $?
cp -r gpurun_out/clock $OUT/ 2>/dev/null
echo done >> $OUT/status.txt
