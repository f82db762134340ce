#!/bin/bash
# r05: the bench line alone on a fresh box (box-to-box spread of one build)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-benchonly}; mkdir -p $OUT
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
echo "bench ok" > $OUT/status.txt
