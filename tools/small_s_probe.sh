set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/small
timeout -k 10 120 python tools/host_overhead.py --shape 2,8,128,64 > gpurun_out/small/host_overhead.log 2>&1 || exit $?
cat gpurun_out/small/host_overhead.log | grep -v "^\["
for sh in 2,8,128,64 2,8,512,64 1,1,512,64 2,8,1024,64; do
  TAG=_$sh SHAPE=$sh bash tools/trace_small.sh || exit $?
  echo "== $sh"; tail -6 gpurun_out/p_$sh/gaps.txt
done
