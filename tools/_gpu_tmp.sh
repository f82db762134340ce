set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
rm -f gpurun_out/status.txt
STEPS="pytest prof" bash tools/gpu_check.sh || exit $?
tail -3 gpurun_out/pytest_gpu.log
bash tools/pmc.sh || exit $?
tail -30 gpurun_out/pmc/summary.txt
