#!/bin/bash
# A/B (r03): explicit sched_group_barrier pipelines for the unsplit dK/dV step (sgb1-4)
# against the shipped iglp_opt(0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/sgb
V=cuda-flash-attention_amd/variants
L=(--lib cuda-flash-attention_amd/lib/libfa2amd.so)
for n in 1 2 3 4; do L+=(--lib $V/sgb$n/libfa2amd.so); done
timeout -k 10 400 python tools/kbench.py --shape 4,16,2048,64 --kernel dkdv --rounds 15 --do ones "${L[@]}" > gpurun_out/sgb/c3.log 2>&1 || exit $?
grep -v "^\[" gpurun_out/sgb/c3.log | grep -v "^{" | grep -v amdgpu.ids
timeout -k 10 400 python tools/kbench.py --shape 2,8,4096,64 --kernel dkdv --rounds 15 --do ones "${L[@]}" > gpurun_out/sgb/s4096.log 2>&1 || exit $?
grep -v "^\[" gpurun_out/sgb/s4096.log | grep -v "^{" | grep -v amdgpu.ids
