#!/bin/bash
# A/B (r03): LLVM scheduler flags on top of the iglp strategies -- exact igrouplp solver
# (es), no clustered low-occupancy rescheduling (nc)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/sflags
V=cuda-flash-attention_amd/variants
L=(--lib cuda-flash-attention_amd/lib/libfa2amd.so --lib $V/es/libfa2amd.so --lib $V/nc/libfa2amd.so)
run() {  # name shape rounds kernels...
  local n=$1 sh=$2 r=$3; shift 3
  local ks=(); for k in "$@"; do ks+=(--kernel $k); done
  timeout -k 10 400 python tools/kbench.py --shape $sh "${ks[@]}" --rounds $r --do ones "${L[@]}" > gpurun_out/sflags/$n.log 2>&1 || exit $?
  grep -v "^\[" gpurun_out/sflags/$n.log | grep -v "^{" | grep -v amdgpu.ids
}
run c3 4,16,2048,64 13 fwd dq dkdv
run c4 8,16,4096,128 9 fwd
run s512 2,8,512,64 21 bwd
