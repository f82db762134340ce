#!/bin/bash
# r04: cost of the forward's restart (a late score spike redoes every query block with the
# rescaling loop): U[0,1) inputs vs one late spiking key, D = 32 / 64 / 128, C3 and small S
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/spike; mkdir -p $OUT
for sh in 4,16,2048,64 2,8,512,64 2,8,2048,32 2,16,2048,128; do
  for inp in rand spike; do
    timeout -k 10 120 python tools/kbench.py --shape $sh --kernel fwd --inputs $inp --rounds 5 --iters 20 \
      > $OUT/fwd_${sh}_$inp.log 2>&1 || exit $?
  done
done
echo done > $OUT/status.txt
