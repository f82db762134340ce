#!/bin/bash
# r04: single-pass backward (BWD_SP) -- parity, then in-process A/B of fa2_backward
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sp; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "single_pass or two_kernel_plan" \
   --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" > $OUT/status.txt
case $rc in 0|1) ;; *) exit $rc;; esac
for sh in 4,16,2048,64 2,8,4096,64; do
  for d in ones randn; do
    timeout -k 10 200 python tools/kbench.py --shape $sh --kernel bwd --kernel stepb --do $d --rounds 9 --iters 20 \
      --variant BWD_SP=0 --variant BWD_SP=1 --variant BWD_SP=2 > $OUT/ab_${sh}_$d.log 2>&1 || exit $?
  done
done
timeout -k 10 200 python tools/kbench.py --shape 64,16,2048,64 --kernel stepb --do ones --rounds 7 --iters 8 \
   --variant BWD_SP=0 --variant BWD_SP=1 --variant BWD_SP=2 > $OUT/ab_c5.log 2>&1 || exit $?
echo ab ok >> $OUT/status.txt
