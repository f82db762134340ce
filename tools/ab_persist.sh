#!/bin/bash
# GPU box: parity of the persistent dK/dV walk, then an in-process A/B against the
# default kernel (DKDV_PERSIST=0/1) at C3, C5 and B4_H16_S4096.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider \
  -k "persistent or backward_split or two_kernel or deterministic" --timeout 120 --timeout-method thread \
  > gpurun_out/ab/persist_tests.log 2>&1 || { tail -30 gpurun_out/ab/persist_tests.log; exit 1; }
tail -2 gpurun_out/ab/persist_tests.log
for sh in ${SHAPES:-4,16,2048,64 4,16,4096,64 64,16,2048,64}; do
  timeout -k 10 300 python tools/kbench.py --shape "$sh" --kernel dkdv --kernel stepb --do ones --rounds ${ROUNDS:-9} \
    --variant DKDV_PERSIST=0 --variant DKDV_PERSIST=1 > gpurun_out/ab/persist_$sh.log 2>&1 || exit $?
  grep -v "^\[" gpurun_out/ab/persist_$sh.log | grep -v "^{" | tail -6
done
