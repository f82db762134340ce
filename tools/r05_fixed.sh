#!/bin/bash
# r05: per-workgroup fixed cost vs per-tile cost of the C3-class kernels.  Same grid (512
# workgroups of 256 rows, D = 64) at 16 / 32 / 64 / 128 tiles per workgroup, plus one
# round (256 workgroups).  T = rounds * (F + tiles * t) separates F from t.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/fixed; mkdir -p $OUT
for sh in 8,16,1024,64 4,16,2048,64 2,16,4096,64 1,16,8192,64 2,16,2048,64; do
  timeout -k 10 120 python tools/kbench.py --shape $sh --kernel fwd --kernel dqd --kernel dkdv --do randn \
     --rounds 5 --iters 20 > $OUT/kb_$sh.log 2>&1 || exit $?
done
echo done > $OUT/status.txt
