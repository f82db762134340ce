#!/bin/bash
# r05: schedule-knob A/Bs of the hand-scheduled loops (exact-result builds: 'epgN' v_exp per
# gap, 'capN' minimum gap issue budget; tools/r05_hs_abl.sh), in-process against the product
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/knobs; mkdir -p $OUT
L=cuda-flash-attention_amd
A=$L/abl
for sh in 4,16,2048,64 2,8,4096,64; do
  timeout -k 10 200 python -u tools/kbench.py --shape $sh --kernel fwd --rounds 7 --iters 20 --lib $L/lib/libfa2amd.so \
     --lib $A/fw_epg3/libfa2amd.so --lib $A/fw_epg4/libfa2amd.so > $OUT/fwd_$sh.log 2>&1 || exit $?
  timeout -k 10 200 python -u tools/kbench.py --shape $sh --kernel dqd --rounds 7 --iters 20 --lib $L/lib/libfa2amd.so \
     --lib $A/dq_epg2/libfa2amd.so --lib $A/dq_cap8/libfa2amd.so --lib $A/dq_cap16/libfa2amd.so > $OUT/dq_$sh.log 2>&1 || exit $?
  timeout -k 10 200 python -u tools/kbench.py --shape $sh --kernel dkdv --rounds 7 --iters 20 --variant DKDV_HS=1 \
     --lib $L/lib/libfa2amd.so --lib $A/dk_epg2/libfa2amd.so --lib $A/dk_cap16/libfa2amd.so --lib $A/dk_cap32/libfa2amd.so \
     > $OUT/dk_$sh.log 2>&1 || exit $?
done
timeout -k 10 200 python -u tools/kbench.py --shape 8,16,4096,128 --kernel fwd --rounds 5 --iters 10 --lib $L/lib/libfa2amd.so \
   --lib $A/fw_epg3/libfa2amd.so > $OUT/fwd_c4.log 2>&1 || exit $?
echo "ab ok" > $OUT/status.txt
