#!/bin/bash
# PMC A/B of library builds on one kernel: tools/pmc_ab.sh <kernel> <shape> <lib>...
# Two counter passes per library (no tracing domains combined with --pmc);
# summary per library in gpurun_out/pmcab/<n>/summary.txt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
K=$1; SH=$2; shift 2
PASSES=(
  "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_VALU_TRANS_F32 SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY"
  "GRBM_GUI_ACTIVE SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_WAVES"
)
n=0
for L in "$@"; do
  n=$((n+1)); OUT=gpurun_out/pmcab/$n; mkdir -p $OUT; echo "$L" > $OUT/lib.txt
  i=0
  for p in "${PASSES[@]}"; do
    i=$((i+1))
    timeout -k 10 200 rocprofv3 --pmc $p -d $OUT/p$i -o run --output-format csv -- \
      python3 tools/kbench.py --shape $SH --kernel $K --lib $L --rounds 1 --iters 3 > $OUT/p$i.log 2>&1 || exit $?
  done
  python3 tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1
done
