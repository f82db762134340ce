#!/bin/bash
# confirmation A/B (r03): iglp_opt(2) on the fused small-grid backward (fz2) vs default
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/iglp5
L=(--lib cuda-flash-attention_amd/lib/libfa2amd.so --lib cuda-flash-attention_amd/variants/fz2/libfa2amd.so)
run() {  # name shape rounds kernel do
  timeout -k 10 400 python tools/kbench.py --shape $2 --kernel $4 --rounds $3 --do $5 "${L[@]}" > gpurun_out/iglp5/$1.log 2>&1 || exit $?
  grep -v "^\[" gpurun_out/iglp5/$1.log | grep -v "^{" | grep -v amdgpu.ids
}
run s512_ones 2,8,512,64 25 bwd ones
run s512_randn 2,8,512,64 25 bwd randn
run s512_step 2,8,512,64 25 step ones
run b4h8_s512 4,8,512,64 21 bwd ones
run d32_s1024 2,8,1024,32 21 bwd ones
run s1024_step 2,8,1024,64 21 step ones
