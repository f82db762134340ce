set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "mfma_shape or golden or forward" > gpurun_out/t_fwd.log 2>&1 || exit $?
for sh in 4,16,2048,64 2,8,4096,64 4,16,2048,32 8,16,2048,64; do
  timeout -k 10 150 python tools/kbench.py --shape $sh --kernel fwd --variant FWD_MF=32 --variant FWD_MF=16 --rounds 9 > gpurun_out/kb10_$sh.log 2>&1 || exit $?
done
