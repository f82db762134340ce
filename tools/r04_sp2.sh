#!/bin/bash
# r04: single-pass backward with Δ from a separate launch (FA2_SP_DEL=0) -- parity, then in-process A/B
# against the two-kernel plan and against the FA2_SP_MID build (part product after the staging loads)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sp2; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "single_pass or two_kernel_plan" \
   --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || exit $?
M=cuda-flash-attention_amd/lib/libfa2amd.so; V=cuda-flash-attention_amd/variants/sp_mid/libfa2amd.so
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/pmid -o run --output-format csv -- python3 tools/kbench.py \
   --shape 4,16,2048,64 --kernel bwd --do ones --rounds 3 --iters 20 --lib $V --variant BWD_SP=1 > $OUT/kb_mid.log 2>&1 || exit $?
for sh in 4,16,2048,64 2,8,4096,64 1,16,8192,64; do
  timeout -k 10 200 python tools/kbench.py --shape $sh --kernel bwd --kernel stepb --do ones --rounds 9 --iters 20 \
    --lib $M --lib $V --variant BWD_SP=0 --variant BWD_SP=1 > $OUT/ab_${sh}.log 2>&1 || exit $?
done
timeout -k 10 200 python tools/kbench.py --shape 64,16,2048,64 --kernel stepb --do ones --rounds 7 --iters 8 \
   --lib $M --lib $V --variant BWD_SP=0 --variant BWD_SP=1 > $OUT/ab_c5.log 2>&1 || exit $?
echo ab ok > $OUT/status.txt
