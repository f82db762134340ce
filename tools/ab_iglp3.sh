#!/bin/bash
# A/B: default scheduler vs iglp_opt(0) on the unsplit dK/dV kernel (ig00) and also
# iglp_opt(1) on the unsplit dQ kernel (ig01), in one process per shape (r03)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/iglp
V=cuda-flash-attention_amd/variants
LIBS=(--lib cuda-flash-attention_amd/lib/libfa2amd.so --lib $V/ig00/libfa2amd.so --lib $V/ig01/libfa2amd.so)
run() {  # name shape rounds kernels...
  local n=$1 sh=$2 r=$3; shift 3
  local ks=(); for k in "$@"; do ks+=(--kernel $k); done
  timeout -k 10 400 python tools/kbench.py --shape $sh "${ks[@]}" --rounds $r --do ones "${LIBS[@]}" > gpurun_out/iglp/$n.log 2>&1 || exit $?
  grep -v "^\[" gpurun_out/iglp/$n.log | grep -v "^{" | grep -v amdgpu.ids
}
run c3_kern 4,16,2048,64 15 dkdv dq
run c3_step 4,16,2048,64 15 step
run s4096 2,8,4096,64 15 step
run c5 64,16,2048,64 5 step
run d32 16,16,2048,32 9 bwd
