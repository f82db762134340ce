#!/bin/bash
# A/B of LLVM's iglp_opt scheduling strategies (0-3) on the backward step bodies (r03)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/iglp
V=cuda-flash-attention_amd/variants
LIBS=(--lib cuda-flash-attention_amd/lib/libfa2amd.so)
for n in 0 1 2 3; do LIBS+=(--lib $V/iglp$n/libfa2amd.so); done
timeout -k 10 400 python tools/kbench.py --shape 4,16,2048,64 --kernel dkdv --kernel dq --rounds 9 --do ones "${LIBS[@]}" > gpurun_out/iglp/c3.log 2>&1 || exit $?
grep -v "^\[" gpurun_out/iglp/c3.log | grep -v "^{" | grep -v amdgpu.ids
timeout -k 10 400 python tools/kbench.py --shape 2,8,1024,64 --kernel bwd --rounds 9 --do ones "${LIBS[@]}" > gpurun_out/iglp/s1024.log 2>&1 || exit $?
grep -v "^\[" gpurun_out/iglp/s1024.log | grep -v "^{" | grep -v amdgpu.ids
