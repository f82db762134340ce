#!/bin/bash
# r05: first GPU run of the hand-scheduled forward: parity tests, then an in-process A/B
# against the compiler-scheduled kernel at C3 and C4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fwd_hs.py \
    "tests/test_gpu_parity.py::test_cupy_face_backward_bitwise_repeatable" "tests/test_gpu_parity.py::test_cupy_face_geometry_fp16" \
    "tests/test_gpu_parity.py::test_cupy_face_geometry_bf16" \
    > gpurun_out/hs_tests.log 2>&1
rc=$?
tail -40 gpurun_out/hs_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/kbench.py --shape 4,16,2048,64 --kernel fwd --variant FWD_HS=0 --variant FWD_HS=1 \
    > gpurun_out/hs_kbench_c3.log 2>&1 && tail -5 gpurun_out/hs_kbench_c3.log &&
timeout -k 10 200 python -u tools/kbench.py --shape 8,16,4096,128 --kernel fwd --variant FWD_HS=0 --variant FWD_HS=1 --rounds 5 --iters 10 \
    > gpurun_out/hs_kbench_c4.log 2>&1 && tail -5 gpurun_out/hs_kbench_c4.log
