#!/bin/bash
# Clock / socket power while each kernel runs alone in a long loop: which kernels run
# at the power cap?  Output: gpurun_out/clock/<kernel>.txt (amd-smi samples)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/clock; mkdir -p $OUT
for kn in ${KERNELS:-fwd dqd dkdv step}; do
  python3 tools/kbench.py --kernel $kn --rounds 400 --iters 100 > $OUT/kb_$kn.log 2>&1 &
  P=$!
  sleep 6
  for i in 1 2 3 4 5; do
    amd-smi metric -g 0 -c -p 2>/dev/null | grep -iE "socket_power|gfx_0|clk" | head -6 >> $OUT/$kn.txt; echo "--" >> $OUT/$kn.txt; sleep 1
  done
  kill $P 2>/dev/null; wait $P 2>/dev/null
done
