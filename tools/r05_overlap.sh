#!/bin/bash
# r05: MFMA / filler overlap probe (tools/microbench/gen_overlap.py), one wave per SIMD
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/overlap
timeout -k 10 120 ./tools/microbench/overlap > gpurun_out/overlap/overlap.log 2>&1
