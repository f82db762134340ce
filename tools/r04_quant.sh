#!/bin/bash
# full grids with a fractional last round of workgroups: split plans with whole rounds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/quant; mkdir -p $OUT
for sh in 3,8,4096,64 6,8,2048,64 5,16,2048,64; do
  timeout -k 10 150 python tools/kbench.py --shape $sh --kernel fwd --kernel dq --kernel dkdv --do ones --rounds 7 --variant "" \
    --variant FWD_KS=2,FWD_WAVES=8,DQ_KS=2,DQ_WAVES=8,DKDV_QS=2,DKDV_WAVES=8 > $OUT/ab_$sh.log 2>&1 || exit $?
done
