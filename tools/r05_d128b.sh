#!/bin/bash
# r05: D = 128 forward schedule A/Bs on the adopted schedule (3 v_exp per gap, spread loads): epg2, epg4, cap16, cap32
# -- in-process against the product
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/d128b; mkdir -p $OUT
L=cuda-flash-attention_amd
A=$L/abl
for sh in 8,16,4096,128 2,16,4096,128 4,16,2048,128; do
  timeout -k 10 250 python -u tools/kbench.py --shape $sh --kernel fwd --rounds 9 --iters 10 --lib $L/lib/libfa2amd.so \
     --lib $A/f8_epg2/libfa2amd.so --lib $A/f8_epg4/libfa2amd.so --lib $A/f8_cap16/libfa2amd.so --lib $A/f8_cap32/libfa2amd.so > $OUT/fwd_$sh.log 2>&1 || exit $?
done
echo "ab ok" > $OUT/status.txt
