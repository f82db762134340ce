set -o pipefail
mkdir -p gpurun_out
for s in 512 1024 2048; do
  timeout -k 10 120 python tools/kbench.py --shape 2,8,$s,64 --kernel step --kernel step2s --kernel step2r --kernel fwd --kernel dqd --kernel dkdv --do ones --rounds 5 > gpurun_out/kb_s$s.log 2>&1 || exit $?
done
