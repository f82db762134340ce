#!/bin/bash
# A/B of MFMA operand-order variants (consecutive MFMAs sharing an operand) in one
# process: usage  tools/ab_energy.sh <variant> [shape kernels...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/energy
V=$1; shift
L=cuda-flash-attention_amd/lib/libfa2amd.so
A=cuda-flash-attention_amd/variants/$V/libfa2amd.so
while [ $# -gt 0 ]; do
  shape=$1; kern=$2; shift 2
  ks=(); for k in ${kern//,/ }; do ks+=(--kernel $k); done
  timeout -k 10 300 python tools/kbench.py --shape $shape "${ks[@]}" --rounds 11 --do ones --lib $L --lib $A > gpurun_out/energy/${V}_${shape//,/_}.log 2>&1 || exit $?
  grep -v "^\[" gpurun_out/energy/${V}_${shape//,/_}.log | grep -v "^{" | grep -v amdgpu.ids
done
