#!/bin/bash
# r04: global-load energy (microbench modes 10/11) and the pipelined dQ loop in the steady-state step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/p3; mkdir -p $OUT
MODES="0 10 11 2" timeout -k 10 120 bash tools/energy_probe.sh || exit $?
cp gpurun_out/energy/m0.* gpurun_out/energy/m10.* gpurun_out/energy/m11.* gpurun_out/energy/m2.* $OUT/
timeout -k 10 250 python tools/kbench.py --shape 4,16,2048,64 --kernel step --do ones --rounds 15 --iters 100 \
   --variant DQ_PIPE=0,DQ_WAVES=8 --variant DQ_PIPE=1,DQ_WAVES=8 > $OUT/step_c3.log 2>&1 || exit $?
timeout -k 10 250 python tools/kbench.py --shape 64,16,2048,64 --kernel step --do ones --rounds 9 --iters 8 \
   --variant DQ_PIPE=0,DQ_WAVES=8 --variant DQ_PIPE=1,DQ_WAVES=8 > $OUT/step_c5.log 2>&1 || exit $?
echo done > $OUT/status.txt
