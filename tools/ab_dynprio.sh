#!/bin/bash
# A/B (r03): s_setprio 1 around the dK/dV step's MFMA phases (dprio) vs shipped
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/dprio
L=(--lib cuda-flash-attention_amd/lib/libfa2amd.so --lib cuda-flash-attention_amd/variants/dprio/libfa2amd.so)
for sh in 4,16,2048,64 2,8,4096,64; do
  timeout -k 10 400 python tools/kbench.py --shape $sh --kernel dkdv --rounds 15 --do ones "${L[@]}" > gpurun_out/dprio/${sh//,/_}.log 2>&1 || exit $?
  grep -v "^\[" gpurun_out/dprio/${sh//,/_}.log | grep -v "^{" | grep -v amdgpu.ids
done
