#!/bin/bash
# A/B (r03, after the scheduling changes): launch plans at the north star's sweep points
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/plans
run() {  # name shape kernel variants...
  local n=$1 sh=$2 k=$3; shift 3
  local vs=(); for v in "$@"; do vs+=(--variant $v); done
  timeout -k 10 400 python tools/kbench.py --shape $sh --kernel $k --rounds 15 --do ones "${vs[@]}" > gpurun_out/plans/$n.log 2>&1 || exit $?
  grep -v "^\[" gpurun_out/plans/$n.log | grep -v "^{" | grep -v amdgpu.ids
}
run fwd_s2048 2,8,2048,64 fwd FWD_KS=0 FWD_KS=1,FWD_WAVES=8 FWD_KS=1,FWD_WAVES=4 FWD_KS=4,FWD_WAVES=8
run fwd_s1024 2,8,1024,64 fwd FWD_KS=0 FWD_KS=2,FWD_WAVES=8 FWD_KS=4,FWD_WAVES=4 FWD_KS=2,FWD_WAVES=4
run fwd_s512 2,8,512,64 fwd FWD_KS=0 FWD_KS=4,FWD_WAVES=8 FWD_KS=2,FWD_WAVES=4
run bwd_s2048 2,8,2048,64 bwd BWD_FUSED_DELTA=0 BWD_FUSED_DELTA=1 BWD_FUSED=0
run bwd_s4096 2,8,4096,64 bwd BWD_FUSED=0 BWD_FUSED=1
run bwd_s1024 2,8,1024,64 bwd BWD_FUSED_DELTA=1 BWD_FUSED_DELTA=0
