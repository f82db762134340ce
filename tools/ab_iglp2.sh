#!/bin/bash
# confirmation A/B: base vs iglp_opt(0) / (1) on the backward steps, more rounds + the step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/iglp
V=cuda-flash-attention_amd/variants
LIBS=(--lib cuda-flash-attention_amd/lib/libfa2amd.so --lib $V/iglp0/libfa2amd.so --lib $V/iglp1/libfa2amd.so)
timeout -k 10 400 python tools/kbench.py --shape 4,16,2048,64 --kernel dkdv --kernel dq --rounds 21 --do ones "${LIBS[@]}" > gpurun_out/iglp/c3b.log 2>&1 || exit $?
grep -v "^\[" gpurun_out/iglp/c3b.log | grep -v "^{" | grep -v amdgpu.ids
timeout -k 10 400 python tools/kbench.py --shape 4,16,2048,64 --kernel step --rounds 15 --do ones "${LIBS[@]}" > gpurun_out/iglp/c3step.log 2>&1 || exit $?
grep -v "^\[" gpurun_out/iglp/c3step.log | grep -v "^{" | grep -v amdgpu.ids
timeout -k 10 400 python tools/kbench.py --shape 2,8,4096,64 --kernel bwd --rounds 15 --do ones "${LIBS[@]}" > gpurun_out/iglp/s4096.log 2>&1 || exit $?
grep -v "^\[" gpurun_out/iglp/s4096.log | grep -v "^{" | grep -v amdgpu.ids
