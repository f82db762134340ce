#!/bin/bash
# r04: single-pass backward parity, first case alone with serialized kernels, then the rest
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sp; mkdir -p $OUT
AMD_SERIALIZE_KERNEL=3 timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x \
   -k "single_pass_backward and B1_H32_S2048_D64 and fp32_parts" --timeout 150 --timeout-method thread \
   -p no:cacheprovider > $OUT/pytest_dbg.log 2>&1
rc=$?; echo "dbg rc=$rc" > $OUT/status.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "single_pass or two_kernel_plan" \
   --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/status.txt
exit $rc
