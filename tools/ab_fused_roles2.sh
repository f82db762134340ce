#!/bin/bash
# confirmation A/B (r03): unsplit roles (FQS = FKS = 1) vs the 2/2 default of grids with
# 4-8 blocks of 32 rows per CU, and the two-kernel plan, fwd + bwd step included
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/froles
run() {  # name shape kernel do
  timeout -k 10 400 python tools/kbench.py --shape $2 --kernel $3 --rounds 15 --do $4 \
    --variant BWD_FNW=0 --variant BWD_FQS=1,BWD_FKS=1 --variant BWD_FUSED=0 > gpurun_out/froles/$1.log 2>&1 || exit $?
  grep -v "^\[" gpurun_out/froles/$1.log | grep -v "^{" | grep -v amdgpu.ids
}
run s2048_ones 2,8,2048,64 bwd ones
run s2048_randn 2,8,2048,64 bwd randn
run s2048_step 2,8,2048,64 step ones
run s2048_d32 2,8,2048,32 bwd ones
run b4h8_s1024 4,8,1024,64 bwd ones
run b1h16_s4096 1,16,4096,64 bwd ones
run s1500 2,8,1500,64 bwd ones
