set -o pipefail
mkdir -p gpurun_out/w4
timeout -k 10 300 python tools/kbench.py --shape 4,16,2048,64 --kernel dkdv --kernel dq --kernel fwd --rounds 9 --variant DKDV_WAVES=8,DQ_WAVES=8,FWD_WAVES=8 --variant DKDV_WAVES=4,DQ_WAVES=4,FWD_WAVES=4 > gpurun_out/w4/kb_c3.log 2>&1 || exit $?
grep -v "^\[" gpurun_out/w4/kb_c3.log | grep -v "^{" | tail -8
timeout -k 10 300 python tools/kbench.py --shape 4,16,2048,64 --kernel step --rounds 9 --variant DKDV_WAVES=8 --variant DKDV_WAVES=4 --variant DKDV_WAVES=4,DQ_WAVES=4 > gpurun_out/w4/kb_step.log 2>&1 || exit $?
grep -v "^\[" gpurun_out/w4/kb_step.log | grep -v "^{" | tail -8
