# GPU box: single-pass backward ablations (variant builds -DSP_ABL=..., tools/build_variant.sh)
# and the owner/sweep split (tools/sp_probe.py).  VARIANTS="sp_a12 ..." SHAPES="4,16,2048,64 ..."
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/ab
V=cuda-flash-attention_amd/variants
LIBS="--lib cuda-flash-attention_amd/lib/libfa2amd.so"
for v in ${VARIANTS}; do LIBS="$LIBS --lib $V/$v/libfa2amd.so"; done
for sh in ${SHAPES:-4,16,2048,64}; do
  timeout -k 10 120 python tools/sp_probe.py --shape $sh > gpurun_out/ab/probe_$sh.log 2>&1 || exit $?
  grep -v "^/opt" gpurun_out/ab/probe_$sh.log
  timeout -k 10 300 python tools/kbench.py --shape $sh --kernel bwd --variant BWD_SP=1 --rounds 5 $LIBS > gpurun_out/ab/sp_$sh.log 2>&1 || exit $?
  grep -v "^\[" gpurun_out/ab/sp_$sh.log | grep -v "^{" | grep -v "^/opt"
done
