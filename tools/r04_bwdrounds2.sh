#!/bin/bash
# the fused small-grid backward's role-split rule (one round of workgroups): parity, A/Bs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/bwdr2; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "fused or backward_split or golden or determin" > $OUT/pytest.log 2>&1 || exit $?
K="--kernel bwd --kernel step --do ones --rounds 9"
timeout -k 10 150 python tools/kbench.py --shape 2,8,1500,64 $K --variant "" --variant BWD_FQS=2,BWD_FKS=2 --variant BWD_FUSED_DELTA=0 > $OUT/ab_1500.log 2>&1 || exit $?
timeout -k 10 150 python tools/kbench.py --shape 3,8,1024,64 $K --variant "" --variant BWD_FQS=2,BWD_FKS=2 --variant BWD_FUSED_DELTA=0 > $OUT/ab_3_8_1024.log 2>&1 || exit $?
timeout -k 10 150 python tools/kbench.py --shape 2,8,1024,64 $K --variant "" > $OUT/ab_1024.log 2>&1 || exit $?
timeout -k 10 150 python tools/kbench.py --shape 2,8,512,64 $K --variant "" > $OUT/ab_512.log 2>&1 || exit $?
Kf="--kernel fwd --kernel step --do ones --rounds 9"
timeout -k 10 150 python tools/kbench.py --shape 2,8,1024,64 $Kf --variant "" --variant FWD_KS=2,FWD_WAVES=8 > $OUT/fab_1024.log 2>&1 || exit $?
timeout -k 10 150 python tools/kbench.py --shape 2,8,512,64 $Kf --variant "" --variant FWD_KS=2,FWD_WAVES=8 --variant FWD_KS=4,FWD_WAVES=8 > $OUT/fab_512.log 2>&1 || exit $?
