#!/bin/bash
# r05: hand-scheduled dQ and dK/dV parity, then A/B of each kernel and the step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bwd_hs.py \
    > gpurun_out/hs4_tests.log 2>&1
rc=$?
tail -15 gpurun_out/hs4_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/kbench.py --shape 4,16,2048,64 --kernel dqd --variant DQ_HS=0 --variant DQ_HS=1 \
    > gpurun_out/hs4_kbench_dq.log 2>&1 && grep median gpurun_out/hs4_kbench_dq.log &&
timeout -k 10 200 python -u tools/kbench.py --shape 4,16,2048,64 --kernel dkdv --variant DKDV_HS=0 --variant DKDV_HS=1 \
    > gpurun_out/hs4_kbench_dkdv.log 2>&1 && grep median gpurun_out/hs4_kbench_dkdv.log &&
timeout -k 10 200 python -u tools/kbench.py --shape 4,16,2048,64 --kernel step --variant FWD_HS=0,DQ_HS=0,DKDV_HS=0 --variant FWD_HS=1,DQ_HS=1,DKDV_HS=1 \
    > gpurun_out/hs4_kbench_step.log 2>&1 && grep median gpurun_out/hs4_kbench_step.log &&
bash tools/r05_hs2.sh
