#!/bin/bash
# D = 32 small-grid plans between the sweep's sizes (forward plans, fused backward roles)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/d32; mkdir -p $OUT
Kf="--kernel fwd --do ones --rounds 9"
Kb="--kernel bwd --do ones --rounds 9"
for sh in 2,8,1500,32 2,8,3000,32 2,8,2048,32 2,8,1024,32; do
  timeout -k 10 150 python tools/kbench.py --shape $sh $Kf --variant "" --variant FWD_KS=2,FWD_WAVES=8 \
    --variant FWD_KS=1,FWD_WAVES=8 --variant FWD_KS=4,FWD_WAVES=8 > $OUT/fwd_$sh.log 2>&1 || exit $?
done
for sh in 2,8,1500,32 3,8,1024,32 2,8,1024,32; do
  timeout -k 10 150 python tools/kbench.py --shape $sh $Kb --variant "" --variant BWD_FQS=2,BWD_FKS=2 \
    --variant BWD_FQS=1,BWD_FKS=1 > $OUT/bwd_$sh.log 2>&1 || exit $?
done
