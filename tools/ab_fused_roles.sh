#!/bin/bash
# A/B (r03, after iglp_opt(2) on the fused backward): role geometry of the fused
# small-grid backward at the north star's small sweep points
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/froles
for sh in 2,8,512,64 2,8,1024,64 2,8,2048,64; do
  timeout -k 10 400 python tools/kbench.py --shape $sh --kernel bwd --rounds 15 --do ones \
    --variant BWD_FNW=0 --variant BWD_FNW=8,BWD_FQS=2,BWD_FKS=2 --variant BWD_FNW=4,BWD_FQS=2,BWD_FKS=2 \
    --variant BWD_FNW=8,BWD_FQS=2,BWD_FKS=4 --variant BWD_FNW=4,BWD_FQS=2,BWD_FKS=4 --variant BWD_FQS=1,BWD_FKS=1 \
    > gpurun_out/froles/${sh//,/_}.log 2>&1 || exit $?
  grep -v "^\[" gpurun_out/froles/${sh//,/_}.log | grep -v "^{" | grep -v amdgpu.ids
done
