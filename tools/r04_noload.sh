#!/bin/bash
# staging-load ablation (timing-only build -DFA2_ABL_NOLOAD: no global loads in the tile stagers)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/noload; mkdir -p $OUT
L=cuda-flash-attention_amd
for sh in 4,16,2048,64; do
  timeout -k 10 200 python tools/kbench.py --shape $sh --kernel fwd --kernel dq --kernel dkdv --kernel bwd --do ones \
    --rounds 7 --lib $L/lib/libfa2amd.so --lib $L/variants/noload/libfa2amd.so --lib $L/variants/noload2/libfa2amd.so > $OUT/ab_$sh.log 2>&1 || exit $?
done
