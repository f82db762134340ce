#!/bin/bash
# r05: phase stamps of the hand-scheduled forward and dQ loops (timing-only builds), loaded and isolated
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/stamps; mkdir -p $OUT
A=cuda-flash-attention_amd/abl
timeout -k 10 120 python tools/stamps_hs.py --lib $A/fw_stamps/libfa2amd.so \
  --shape 4,16,2048,64 --shape 1,1,2048,64 --shape 1,16,2048,64 --shape 8,16,4096,128 > $OUT/fwd.log 2>&1 &&
timeout -k 10 120 python tools/stamps_hs.py --kernel dq --lib $A/dq_stamps/libfa2amd.so \
  --shape 4,16,2048,64 --shape 1,1,2048,64 > $OUT/dq.log 2>&1 || exit $?
echo done > $OUT/status.txt
