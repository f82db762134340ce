#!/bin/bash
# r04 final check, part A: smoke and the whole -m gpu suite on the committed head
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04fa; mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
echo "smoke ok" > $OUT/status.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/status.txt; exit $rc
