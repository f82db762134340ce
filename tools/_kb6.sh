set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_all.log 2>&1 || exit $?
L=cuda-flash-attention_amd/lib/libfa2amd.so; P=cuda-flash-attention_amd/variants/prev/libfa2amd.so
for sh in 4,16,2048,64 2,8,4096,64 2,8,512,64 4,16,2048,32 1,16,2048,128; do
  timeout -k 10 150 python tools/kbench.py --shape $sh --kernel dkdv --kernel stepb --lib $P --lib $L --do randn --rounds 7 > gpurun_out/kb6_$sh.log 2>&1 || exit $?
done
