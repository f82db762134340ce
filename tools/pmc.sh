#!/bin/bash
# rocprofv3 PMC passes over a short bench run (one counter group per pass, no
# tracing domains combined with --pmc).  Output: gpurun_out/pmc/<pass>/...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmc
mkdir -p $OUT
ARGS="${BENCH_ARGS:---steps 5 --warmup 2 --warmup-ms 0 --no-cpu-baseline --no-extras}"
PASSES=(
  "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_VALU_TRANS_F32 SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY"
  "FETCH_SIZE GRBM_GUI_ACTIVE"
  "WRITE_SIZE SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_ANY"
)
i=0
for p in "${PASSES[@]}"; do
  i=$((i+1))
  echo "== pass $i: $p" >> $OUT/status.txt
  timeout -k 10 300 rocprofv3 --pmc $p -d $OUT/p$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc" >> $OUT/status.txt
  [ $rc -ne 0 ] && exit $rc
done
# the build id of the library the passes profiled: bench.py reports traffic only while
# the library it loads has the same one (a rebuilt kernel cannot inherit old figures)
BID=$(python3 -c "import sys; sys.path.insert(0, 'cuda-flash-attention_amd'); import fa2amd; print(fa2amd.build_id())")
PMC_META='{"S": 2048, "D": 64, "heads": 64, "workload": "B4_H16_S2048_D64 fp16, bench.py --steps 5 --warmup 2", "source": "tools/pmc.sh", "build_id": "'$BID'"}' python3 tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1
echo done >> $OUT/status.txt
