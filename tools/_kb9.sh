set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_all.log 2>&1 || exit $?
L=cuda-flash-attention_amd/lib/libfa2amd.so; P=cuda-flash-attention_amd/variants/prev/libfa2amd.so
for sh in 8,16,4096,128 4,16,2048,64 2,8,512,64 2,8,1024,64 2,8,2048,64 1,16,2048,128; do
  timeout -k 10 150 python tools/kbench.py --shape $sh --kernel fwd --lib $P --lib $L --rounds 9 > gpurun_out/kb9_$sh.log 2>&1 || exit $?
done
