#!/bin/bash
# A/B (r03): iglp_opt on one forward region at D = 64 (QK^T only / PV only), on the whole
# dK/dV step once instead of per 32-query half, and on the fused small-grid backward
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/iglp4
V=cuda-flash-attention_amd/variants
B=cuda-flash-attention_amd/lib/libfa2amd.so
run() {  # name shape rounds kernel libs...
  local n=$1 sh=$2 r=$3 k=$4; shift 4
  local L=(--lib $B); for v in "$@"; do L+=(--lib $V/$v/libfa2amd.so); done
  timeout -k 10 400 python tools/kbench.py --shape $sh --kernel $k --rounds $r --do ones "${L[@]}" > gpurun_out/iglp4/$n.log 2>&1 || exit $?
  grep -v "^\[" gpurun_out/iglp4/$n.log | grep -v "^{" | grep -v amdgpu.ids
}
run fwd_c3 4,16,2048,64 15 fwd fq0 fp0
run dkdv_c3 4,16,2048,64 15 dkdv d1
run bwd_s512 2,8,512,64 21 bwd fz1 fz2
run bwd_s1024 2,8,1024,64 21 bwd fz1 fz2
run bwd_s2048 2,8,2048,64 15 bwd fz1 fz2
