set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_all.log 2>&1 || exit $?
L=cuda-flash-attention_amd/lib/libfa2amd.so; P=cuda-flash-attention_amd/variants/prev/libfa2amd.so
for sh in 4,16,2048,64 2,8,4096,64 8,16,4096,128 2,8,512,64; do
  timeout -k 10 200 python tools/kbench.py --shape $sh --kernel fwd --kernel dqd --kernel step --lib $P --lib $L --do ones --rounds 7 > gpurun_out/kb11_$sh.log 2>&1 || exit $?
done
