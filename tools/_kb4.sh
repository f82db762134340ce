set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_all.log 2>&1 || exit $?
for sh in 2,8,512,64 2,8,1024,64 2,8,2048,64; do
  timeout -k 10 150 python tools/kbench.py --shape $sh --kernel stepb --kernel bwd --variant BWD_FNW=8 --variant BWD_FNW=4 --variant BWD_FNW=4,BWD_FKS=2 --do ones --rounds 5 > gpurun_out/kb4_$sh.log 2>&1 || exit $?
done
L=cuda-flash-attention_amd/lib/libfa2amd.so; P=cuda-flash-attention_amd/variants/prev/libfa2amd.so
for sh in 4,16,2048,64 2,8,512,64; do
  timeout -k 10 150 python tools/kbench.py --shape $sh --kernel step --kernel stepb --lib $P --lib $L --do ones --rounds 5 > gpurun_out/kb4b_$sh.log 2>&1 || exit $?
done
