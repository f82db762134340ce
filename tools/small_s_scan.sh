#!/bin/bash
# GPU box: forward / backward kernel times at small S across head counts (is a
# small-grid launch bound by its per-workgroup chain or by the chip?).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/small
for sh in ${SHAPES:-1,1,512,64 1,4,512,64 2,8,512,64 4,16,512,64 2,8,256,64 2,8,128,64 1,1,1024,64 2,8,1024,64}; do
  timeout -k 10 200 python tools/kbench.py --shape "$sh" --kernel fwd --kernel bwd --kernel stepb --do ones --rounds 7 \
    > gpurun_out/small/scan_$sh.log 2>&1 || exit $?
  echo "== $sh"; grep -v "^\[" gpurun_out/small/scan_$sh.log | grep -v "^{" | tail -3
done
