#!/bin/bash
# r05: where the hand-scheduled forward's loop time goes: timing-only ablation builds
# (tools/r05_hs_abl.sh) against the product build in one process at C3 and C4; then the
# PMC passes of the bench step (tools/pmc.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=cuda-flash-attention_amd
LIBS="--lib $L/lib/libfa2amd.so"
for v in nobar nostage noexp nosm nolds; do LIBS="$LIBS --lib $L/abl/$v/libfa2amd.so"; done
timeout -k 10 300 python -u tools/kbench.py --shape 4,16,2048,64 --kernel fwd $LIBS > gpurun_out/abl_c3.log 2>&1 &&
grep "median" gpurun_out/abl_c3.log &&
timeout -k 10 300 python -u tools/kbench.py --shape 8,16,4096,128 --kernel fwd $LIBS --rounds 5 --iters 10 > gpurun_out/abl_c4.log 2>&1 &&
grep "median" gpurun_out/abl_c4.log &&
timeout -k 10 600 bash tools/pmc.sh && grep -A30 "fa2_fwd_hs" gpurun_out/pmc/summary.txt | head -40
