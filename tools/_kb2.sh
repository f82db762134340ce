set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fused_launch or backward_split" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_fused.log 2>&1 || exit $?
for sh in 2,8,512,64 2,8,1024,64 2,8,2048,64 2,8,4096,64 4,16,2048,64; do
  timeout -k 10 120 python tools/kbench.py --shape $sh --kernel stepb --kernel bwd --variant BWD_FUSED=0 --variant BWD_FUSED=1 --do ones --rounds 5 > gpurun_out/kb2_$sh.log 2>&1 || exit $?
done
