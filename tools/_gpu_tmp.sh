set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
FA2_BENCH_REHEARSE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --no-cpu-baseline > gpurun_out/bench2.log 2>&1 || { echo "bench2 rc=$?"; tail -20 gpurun_out/bench2.log; exit 1; }
grep '^{' gpurun_out/bench2.log
