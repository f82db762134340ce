#!/bin/bash
# r05: workgroup time vs how many workgroups share the chip.  The hand-scheduled kernels
# forced on (FWD_HS / DQ_HS / DKDV_HS = 1) at S = 2048, D = 64 with 8, 32, 128, 256 (one
# round) and 512 (C3, two rounds) workgroups: an isolated workgroup's time against the
# schedule's estimate separates in-CU stalls from chip-level limits (clock, L2, HBM).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/occ; mkdir -p $OUT
for sh in 1,1,2048,64 1,4,2048,64 1,16,2048,64 2,16,2048,64 4,16,2048,64; do
  timeout -k 10 120 python tools/kbench.py --shape $sh --kernel fwd --kernel dqd --kernel dkdv --do randn \
     --variant FWD_HS=1,DQ_HS=1,DKDV_HS=1 --rounds 5 --iters 20 > $OUT/kb_$sh.log 2>&1 || exit $?
done
echo done > $OUT/status.txt
