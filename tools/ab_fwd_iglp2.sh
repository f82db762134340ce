#!/bin/bash
# confirmation A/B at D = 128: iglp_opt(0) / (1) on the forward's QK^T and PV regions (r03)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/figlp
V=cuda-flash-attention_amd/variants
LIBS=(--lib cuda-flash-attention_amd/lib/libfa2amd.so --lib $V/fig0/libfa2amd.so --lib $V/fig1/libfa2amd.so)
for sh in 8,16,4096,128 4,16,2048,128 4,16,2048,64; do
  timeout -k 10 400 python tools/kbench.py --shape $sh --kernel fwd --rounds 21 --do ones "${LIBS[@]}" > gpurun_out/figlp/b_${sh//,/_}.log 2>&1 || exit $?
  grep -v "^\[" gpurun_out/figlp/b_${sh//,/_}.log | grep -v "^{" | grep -v amdgpu.ids
done
