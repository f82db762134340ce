#!/bin/bash
# r04: where the single-pass backward's time goes at C3: per-kernel durations of ablation builds
#   sp_abl1  = no dQ product and no dS image writes (the dK/dV frame + per-step Δ)
#   sp_abl2  = product computed, part stores dropped
#   sp_nodel = Δ from a separate fa2_delta launch, four staging waves
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/spab; mkdir -p $OUT
V=cuda-flash-attention_amd/variants
for l in main sp_abl1 sp_abl2 sp_nodel; do
  if [ $l = main ]; then lib=cuda-flash-attention_amd/lib/libfa2amd.so; else lib=$V/$l/libfa2amd.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/p_$l -o run --output-format csv -- python3 tools/kbench.py \
     --shape 4,16,2048,64 --kernel bwd --do ones --rounds 3 --iters 20 --lib $lib --variant BWD_SP=1 > $OUT/kb_$l.log 2>&1 || exit $?
  f=$(find $OUT/p_$l -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/stats_$l.csv
done
echo done > $OUT/status.txt
