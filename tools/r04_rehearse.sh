#!/bin/bash
# the N > 1 bench path rehearsed on one GPU: 2 ranks over gloo, both on cuda:0
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/rehearse; mkdir -p $OUT
FA2_BENCH_REHEARSE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 10 --warmup 3 > $OUT/bench2.json 2> $OUT/bench2.err || exit $?
