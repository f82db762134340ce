#!/bin/bash
# GPU-box check: smoke -> pytest -m gpu -> bench -> rocprofv3 kernel stats.
# Each GPU step has its own time limit; a crash/abort/timeout ends the script
# (exit codes 124/134/137/139 or negative), a plain test failure (1) does not.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
STEPS="${STEPS:-smoke pytest bench prof}"
fatal() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >> $OUT/status.txt
  timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $OUT/status.txt
  if fatal $rc; then echo "fatal rc=$rc in $name, stopping" >> $OUT/status.txt; exit $rc; fi
  return $rc
}
for s in $STEPS; do
  case $s in
    smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    pytest) run pytest_gpu 1200 python -m pytest tests -m gpu -q --timeout 300 -p no:cacheprovider ${PYTEST_ARGS} ;;
    bench)  run bench 600 python bench.py ${BENCH_ARGS} ;;
    prof)   run prof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extras --steps 50 --warmup 20 ;;
  esac
done
echo done >> $OUT/status.txt
