#!/bin/bash
# r05: hand-scheduled dQ parity + A/B, then the forward ablations and the PMC passes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bwd_hs.py \
    > gpurun_out/hs3_tests.log 2>&1
rc=$?
tail -25 gpurun_out/hs3_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/kbench.py --shape 4,16,2048,64 --kernel dqd --variant DQ_HS=0 --variant DQ_HS=1 \
    > gpurun_out/hs3_kbench_dq.log 2>&1 && grep median gpurun_out/hs3_kbench_dq.log &&
timeout -k 10 200 python -u tools/kbench.py --shape 4,16,2048,64 --kernel step --variant FWD_HS=0,DQ_HS=0 --variant FWD_HS=1,DQ_HS=1 \
    > gpurun_out/hs3_kbench_step.log 2>&1 && grep median gpurun_out/hs3_kbench_step.log &&
bash tools/r05_hs2.sh
