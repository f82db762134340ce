#!/bin/bash
# A/B (r03): iglp strategy per role of the fused small-grid backward (default: 2 on both)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/friglp
V=cuda-flash-attention_amd/variants
L=(--lib cuda-flash-attention_amd/lib/libfa2amd.so)
for n in dk2dqn dkndq2 dk2dq0 dk0dq2; do L+=(--lib $V/$n/libfa2amd.so); done
for sh in 2,8,512,64 2,8,1024,64 2,8,2048,64; do
  timeout -k 10 400 python tools/kbench.py --shape $sh --kernel bwd --rounds 15 --do ones "${L[@]}" > gpurun_out/friglp/${sh//,/_}.log 2>&1 || exit $?
  grep -v "^\[" gpurun_out/friglp/${sh//,/_}.log | grep -v "^{" | grep -v amdgpu.ids
done
