#!/bin/bash
# r04: power of the C4 forward and the S = 4096 step; kernel traces of the small-S steps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/p2; mkdir -p $OUT
timeout -k 10 120 python tools/power_probe.py --shape 8,16,4096,128 --kernel fwd --seconds 4 > $OUT/c4_power.log 2>&1 || exit $?
timeout -k 10 120 python tools/power_probe.py --shape 2,8,4096,64 --kernel fwd --kernel step --seconds 4 > $OUT/s4096_power.log 2>&1 || exit $?
timeout -k 10 120 python tools/power_probe.py --shape 2,8,512,64 --kernel step --seconds 4 > $OUT/s512_power.log 2>&1 || exit $?
for s in 512 1024; do
  TAG=$s SHAPE=2,8,$s,64 timeout -k 10 250 bash tools/trace_small.sh || exit $?
  cp gpurun_out/p$s/gaps.txt $OUT/trace_$s.txt
done
echo done > $OUT/status.txt
