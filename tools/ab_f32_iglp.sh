#!/bin/bash
# A/B (r03): iglp_opt strategies 0-3 on the exact-fp32 kernels at C2 (B2_H8_S512_D64)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/f32ig
V=cuda-flash-attention_amd/variants
L=(--lib cuda-flash-attention_amd/lib/libfa2amd.so)
for n in 0 1 2 3; do L+=(--lib $V/f32ig$n/libfa2amd.so); done
timeout -k 10 400 python tools/kbench.py --shape 2,8,512,64 --precision fp32 --kernel fwd --kernel bwd --rounds 15 --do ones "${L[@]}" > gpurun_out/f32ig/c2.log 2>&1 || exit $?
grep -v "^\[" gpurun_out/f32ig/c2.log | grep -v "^{" | grep -v amdgpu.ids
