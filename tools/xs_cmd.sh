set -o pipefail
mkdir -p gpurun_out/xs
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "key_split or cross_workgroup" > gpurun_out/xs/tests.log 2>&1
rc=$?; tail -5 gpurun_out/xs/tests.log; [ $rc -ne 0 ] && exit $rc
for S in 512 1024; do
timeout -k 10 300 python tools/kbench.py --shape 2,8,$S,64 --kernel fwd --rounds 9 --lib cuda-flash-attention_amd/lib/libfa2amd.so --lib cuda-flash-attention_amd/variants/xsabl/libfa2amd.so --variant FWD_KS=0 --variant FWD_KS=4,FWD_WAVES=8 --variant FWD_KS=4,FWD_WAVES=8,FWD_XS=2 > gpurun_out/xs/kb_$S.log 2>&1 || exit $?
grep -v "^\[" gpurun_out/xs/kb_$S.log | tail -8
done
