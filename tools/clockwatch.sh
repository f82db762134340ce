#!/bin/bash
# Sample GPU clock / power while a kbench step loop runs (is the workload power-capped?)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/clock; mkdir -p $OUT
(for i in $(seq 1 12); do amd-smi metric -g 0 -c -p 2>/dev/null | grep -iE "gfx_0|socket_power|clk:|current_socket|GFX_0" | head -8 >> $OUT/smi.txt; echo "--" >> $OUT/smi.txt; sleep 1; done) &
W=$!
timeout -k 10 60 python3 tools/kbench.py --kernel step --rounds 40 --iters 200 > $OUT/kb.log 2>&1
wait $W
