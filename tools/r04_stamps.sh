#!/bin/bash
# r04: per-workgroup phase stamps of the small-grid forward (timing-only build)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/stamps; mkdir -p $OUT
timeout -k 10 200 python tools/stamps_small.py --lib cuda-flash-attention_amd/variants/stamps/libfa2amd.so \
  > $OUT/fwd.log 2>&1 || exit $?
echo done > $OUT/status.txt
