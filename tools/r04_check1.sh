#!/bin/bash
# r04 first GPU check: full -m gpu suite, fp32 backward A/B against the r03 build,
# host-API wall and CPU time (condition-variable D2H thread vs r03's yield spin).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04c1
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" > $OUT/status.txt
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python tools/kbench_fp32.py --lib cuda-flash-attention_amd/lib/libfa2amd.so \
    --lib cuda-flash-attention_amd/variants/r03/libfa2amd.so --shape 2,8,512,64 --shape 2,8,512,32 \
    --shape 2,8,512,128 --shape 8,16,2048,64 --shape 2,4,1000,64 > $OUT/kbench_fp32.log 2>&1 || exit $?
echo "kbench ok" >> $OUT/status.txt
for lib in cuda-flash-attention_amd/lib/libfa2amd.so cuda-flash-attention_amd/variants/r03/libfa2amd.so; do
  timeout -k 10 300 python tools/host_api_probe.py --c5-only --shards-on-device0 8 --lib $lib \
      > $OUT/host_probe_$(basename $(dirname $lib)).log 2>&1 || exit $?
done
echo "done" >> $OUT/status.txt
