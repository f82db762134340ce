#!/bin/bash
# r05: timing-only ablations of the three hand-scheduled loops at C3 (tools/r05_hs_abl.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=cuda-flash-attention_amd
lib() { local s="--lib $L/lib/libfa2amd.so"; for v in "$@"; do s="$s --lib $L/abl/$v/libfa2amd.so"; done; echo $s; }
timeout -k 10 300 python -u tools/kbench.py --shape 4,16,2048,64 --kernel dqd $(lib dq_nowait dq_nostage dq_nosm dq_nolds dq_nomfma) \
    > gpurun_out/abl5_dq.log 2>&1 && grep median gpurun_out/abl5_dq.log &&
timeout -k 10 300 python -u tools/kbench.py --shape 4,16,2048,64 --kernel dkdv $(lib dk_nowait dk_nostage dk_nosm dk_nolds dk_nomfma) \
    > gpurun_out/abl5_dk.log 2>&1 && grep median gpurun_out/abl5_dk.log &&
timeout -k 10 300 python -u tools/kbench.py --shape 4,16,2048,64 --kernel fwd $(lib fw_nowait fw_nomfma) \
    > gpurun_out/abl5_fw.log 2>&1 && grep median gpurun_out/abl5_fw.log
