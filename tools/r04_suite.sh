#!/bin/bash
# one more fresh-box run of the whole GPU suite (flakiness check) and the bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/suite; mkdir -p $OUT
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 240 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
