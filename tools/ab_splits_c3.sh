#!/bin/bash
# A/B of the small-grid split plans forced onto the C3 grid (r03)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/splits
timeout -k 10 300 python tools/kbench.py --shape 4,16,2048,64 --kernel fwd --rounds 9 --do ones --variant FWD_KS=1 --variant FWD_KS=2,FWD_WAVES=8 > gpurun_out/splits/fwd.log 2>&1 || exit $?
timeout -k 10 300 python tools/kbench.py --shape 4,16,2048,64 --kernel dq --kernel dkdv --rounds 9 --do ones --variant DQ_KS=1,DKDV_QS=1 --variant DQ_KS=2,DQ_WAVES=8,DKDV_QS=2,DKDV_WAVES=8 > gpurun_out/splits/bwd.log 2>&1 || exit $?
timeout -k 10 300 python tools/kbench.py --shape 4,16,2048,64 --kernel bwd --rounds 9 --do ones --variant BWD_FUSED=0 --variant BWD_FUSED=1 > gpurun_out/splits/fused.log 2>&1 || exit $?
for f in fwd bwd fused; do grep -v "^\[" gpurun_out/splits/$f.log | grep -v "^{" | grep -v amdgpu.ids; done
