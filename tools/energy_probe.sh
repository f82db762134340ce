#!/bin/bash
# Socket power while each tools/microbench/energy.hip mode runs alone (see its header).
# Output: gpurun_out/energy/<mode>.json lines {mode, seconds, wave_instr, ...} + power samples
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/energy; mkdir -p $OUT
B=tools/microbench/energy
for m in ${MODES:-0 1 2 3 4 5 6 7 8 9 10 11}; do
  timeout -k 5 30 $B $m 5 > $OUT/m$m.json 2>&1 &
  P=$!
  sleep 1.5
  for i in $(seq 1 10); do
    amd-smi metric -g 0 -p -c 2>/dev/null | grep -E "SOCKET_POWER|^ +CLK:" | head -2 | tr '\n' ' ' >> $OUT/m$m.pw; echo >> $OUT/m$m.pw
    sleep 0.25
  done
  wait $P || exit $?
  sleep 1
done
echo done > $OUT/status.txt
