#!/bin/bash
# confirmation A/B (r03): fused dK/dV role under strategy 0 when its queries are unsplit
# (new lib) vs strategy 2 on both roles (variants/prev: the previous build)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/fdk0
L=(--lib cuda-flash-attention_amd/variants/prev/libfa2amd.so --lib cuda-flash-attention_amd/lib/libfa2amd.so)
for sh in 2,8,2048,64 2,8,1500,64 4,8,1024,64 2,8,2048,32 2,8,512,64; do
  timeout -k 10 400 python tools/kbench.py --shape $sh --kernel bwd --rounds 15 --do ones "${L[@]}" > gpurun_out/fdk0/${sh//,/_}.log 2>&1 || exit $?
  grep -v "^\[" gpurun_out/fdk0/${sh//,/_}.log | grep -v "^{" | grep -v amdgpu.ids
done
