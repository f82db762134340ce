#!/bin/bash
# r04 forward plan change: parity (forced-plan tests), then in-process A/Bs of the old
# rule's plans against the new defaults
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/nkb2; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "key_split or shapes_vs_oracle or forward_golden" > $OUT/pytest.log 2>&1 || exit $?
K="--kernel fwd --kernel step --do ones --rounds 9"
timeout -k 10 150 python tools/kbench.py --shape 2,8,512,64 $K --variant "" --variant FWD_NKB=2 > $OUT/ab_512.log 2>&1 || exit $?
timeout -k 10 150 python tools/kbench.py --shape 2,8,1500,64 $K --variant "" --variant FWD_KS=4,FWD_WAVES=8 > $OUT/ab_1500.log 2>&1 || exit $?
timeout -k 10 150 python tools/kbench.py --shape 2,8,3000,64 $K --variant "" --variant FWD_KS=2,FWD_WAVES=8 > $OUT/ab_3000.log 2>&1 || exit $?
timeout -k 10 150 python tools/kbench.py --shape 3,8,2048,64 $K --variant "" --variant FWD_KS=2,FWD_WAVES=8 > $OUT/ab_3_8_2048.log 2>&1 || exit $?
timeout -k 10 150 python tools/kbench.py --shape 2,8,2048,64 $K --variant "" --variant FWD_NKB=1 > $OUT/ab_2048.log 2>&1 || exit $?
timeout -k 10 150 python tools/kbench.py --shape 2,8,1024,64 $K --variant "" > $OUT/ab_1024.log 2>&1 || exit $?
