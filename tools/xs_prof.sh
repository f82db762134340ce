#!/bin/bash
# rocprofv3 kernel durations of the FWD_XS experiment (r03): B2_H8 S = 512 / 1024 forward,
# default plan, KS = 4 at 8 waves, XS = 2, and XS = 2 without the merge (timing-only build)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
L=cuda-flash-attention_amd/lib/libfa2amd.so
A=cuda-flash-attention_amd/variants/xsabl/libfa2amd.so
n=0; mkdir -p gpurun_out/xs
for S in 512 1024; do
  for spec in "$L|FWD_KS=0" "$L|FWD_KS=4,FWD_WAVES=8" "$L|FWD_KS=4,FWD_WAVES=8,FWD_XS=2" "$A|FWD_KS=4,FWD_WAVES=8,FWD_XS=2"; do
    n=$((n+1)); lib=${spec%%|*}; var=${spec#*|}
    timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/xs/prof_$n -o run --output-format csv -- \
      python3 tools/kbench.py --shape 2,8,$S,64 --kernel fwd --rounds 3 --iters 50 --lib $lib --variant $var \
      > gpurun_out/xs/prof_$n.log 2>&1 || exit $?
    f=$(find gpurun_out/xs/prof_$n -name "*kernel_stats.csv" | head -1)
    echo "S=$S $(basename $(dirname $(dirname $lib)))/$(basename $(dirname $lib)) $var: $(grep fa2_fwd $f | cut -d, -f1-5 | cut -c1-200)"
  done
done
