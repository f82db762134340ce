#!/bin/bash
# r05: timing-only ablation (results invalid): the forward loop without its per-tile barrier --
# the upper bound of what fewer barriers could save
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/nobar; mkdir -p $OUT
L=cuda-flash-attention_amd
for sh in 4,16,2048,64 8,16,4096,128; do
  timeout -k 10 250 python -u tools/kbench.py --shape $sh --kernel fwd --rounds 7 --iters 10 --lib $L/lib/libfa2amd.so \
     --lib $L/abl/fw_nobar/libfa2amd.so > $OUT/fwd_$sh.log 2>&1 || exit $?
done
echo "ab ok" > $OUT/status.txt
