#!/bin/bash
# backward plans on small grids between the sweep's sizes: one round of workgroups or two
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/bwdr; mkdir -p $OUT
K="--kernel bwd --do ones --rounds 9"
timeout -k 10 150 python tools/kbench.py --shape 2,8,1500,64 $K --variant "" --variant BWD_FQS=1,BWD_FKS=1 --variant BWD_FUSED=0 > $OUT/ab_1500.log 2>&1 || exit $?
timeout -k 10 150 python tools/kbench.py --shape 2,8,3000,64 $K --variant "" --variant BWD_FUSED=0 --variant BWD_FQS=2,BWD_FKS=2 > $OUT/ab_3000.log 2>&1 || exit $?
timeout -k 10 150 python tools/kbench.py --shape 3,8,2048,64 $K --variant "" --variant BWD_FUSED=0 --variant BWD_FQS=2,BWD_FKS=2 > $OUT/ab_3_8_2048.log 2>&1 || exit $?
timeout -k 10 150 python tools/kbench.py --shape 2,8,1024,64 $K --variant "" --variant BWD_FQS=1,BWD_FKS=1 > $OUT/ab_1024.log 2>&1 || exit $?
timeout -k 10 150 python tools/kbench.py --shape 3,8,1024,64 $K --variant "" --variant BWD_FQS=1,BWD_FKS=1 --variant BWD_FUSED=0 > $OUT/ab_3_8_1024.log 2>&1 || exit $?
