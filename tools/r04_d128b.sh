#!/bin/bash
# D = 128 small-grid defaults after the r04 wave-count change: parity, then A/Bs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/d128b; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "128 or shapes_vs_oracle or golden or cli" > $OUT/pytest.log 2>&1 || exit $?
for sh in 2,8,512,128 2,8,1500,128 2,8,2048,128; do
  timeout -k 10 150 python tools/kbench.py --shape $sh --kernel fwd --kernel dkdv --kernel bwd --do ones --rounds 7 --variant "" \
    --variant FWD_WAVES=2,DKDV_WAVES=2 > $OUT/ab_$sh.log 2>&1 || exit $?
done
