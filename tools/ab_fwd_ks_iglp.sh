#!/bin/bash
# A/B (r03): iglp_opt strategies 0-3 on the key-split (small-grid) forward instances
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/fk
V=cuda-flash-attention_amd/variants
L=(--lib cuda-flash-attention_amd/lib/libfa2amd.so)
for n in 0 1 2 3; do L+=(--lib $V/fk$n/libfa2amd.so); done
for sh in 2,8,512,64 2,8,1024,64 2,8,2048,64 2,8,1024,32; do
  timeout -k 10 400 python tools/kbench.py --shape $sh --kernel fwd --rounds 21 --do ones "${L[@]}" > gpurun_out/fk/${sh//,/_}.log 2>&1 || exit $?
  grep -v "^\[" gpurun_out/fk/${sh//,/_}.log | grep -v "^{" | grep -v amdgpu.ids
done
