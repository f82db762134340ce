#!/bin/bash
# r05: phase stamps of timing-only ablation builds (one instruction class dropped each):
# which class costs how many cycles in which phase, at C3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/stabl; mkdir -p $OUT
A=cuda-flash-attention_amd/abl
for v in fw_stamps fw_st_noexp fw_st_nosm fw_st_nostage fw_st_nolds fw_st_nomfma; do
  timeout -k 10 120 python tools/stamps_hs.py --lib $A/$v/libfa2amd.so --shape 4,16,2048,64 > $OUT/$v.log 2>&1 || exit $?
done
for v in dq_stamps dq_st_nosm dq_st_nostage dq_st_nomfma; do
  timeout -k 10 120 python tools/stamps_hs.py --kernel dq --lib $A/$v/libfa2amd.so --shape 4,16,2048,64 > $OUT/$v.log 2>&1 || exit $?
done
echo done > $OUT/status.txt
