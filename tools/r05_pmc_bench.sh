#!/bin/bash
# r05: PMC passes of the current build (tools/pmc.sh), then its bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-pmcb}; mkdir -p $OUT
timeout -k 10 400 bash tools/pmc.sh || exit $?
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
echo "pmc + bench ok" > $OUT/status.txt
