#!/bin/bash
# A/B: LLVM iglp_opt strategies 0-3 on the forward's QK^T and PV regions (r03)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/figlp
V=cuda-flash-attention_amd/variants
LIBS=(--lib cuda-flash-attention_amd/lib/libfa2amd.so)
for n in 0 1 2 3; do LIBS+=(--lib $V/fig$n/libfa2amd.so); done
for sh in 4,16,2048,64 8,16,4096,128 2,8,1024,64; do
  timeout -k 10 400 python tools/kbench.py --shape $sh --kernel fwd --rounds 11 --do ones "${LIBS[@]}" > gpurun_out/figlp/${sh//,/_}.log 2>&1 || exit $?
  grep -v "^\[" gpurun_out/figlp/${sh//,/_}.log | grep -v "^{" | grep -v amdgpu.ids
done
