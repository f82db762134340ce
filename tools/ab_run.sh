#!/bin/bash
# GPU box: A/B alternate libfa2amd.so builds (tools/build_variant.sh) against the
# default one in one process per shape, after checking their outputs against it.
#   VARIANTS="fast1 fast2" SHAPES="4,16,2048,64 2,8,4096,64" KERNELS="fwd stepb" bash tools/ab_run.sh
# Logs: gpurun_out/ab/<tag>_equal.log, gpurun_out/ab/<tag>_<shape>.log (TAG, default "ab").
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
TAG=${TAG:-ab}
L0=cuda-flash-attention_amd/lib/libfa2amd.so
LIBS=()
for v in ${VARIANTS}; do LIBS+=("cuda-flash-attention_amd/variants/$v/libfa2amd.so"); done
[ ${#LIBS[@]} -gt 0 ] || { echo "VARIANTS is empty"; exit 2; }
timeout -k 10 120 python tools/lib_equal.py "${LIBS[@]}" --shape 4,16,2048,64 --shape 1,2,300,64 --shape 2,3,128,32 \
  > gpurun_out/ab/${TAG}_equal.log 2>&1
rc=$?; echo "equal rc=$rc"; tail -8 gpurun_out/ab/${TAG}_equal.log
case $rc in 0|1) ;; *) exit $rc;; esac  # 1: outputs differ (reported), anything else: stop
KARGS=(); for k in ${KERNELS:-fwd stepb}; do KARGS+=(--kernel "$k"); done
LARGS=(--lib "$L0"); for l in "${LIBS[@]}"; do LARGS+=(--lib "$l"); done
for sh in ${SHAPES:-4,16,2048,64}; do
  timeout -k 10 300 python tools/kbench.py --shape "$sh" "${KARGS[@]}" --do ones --rounds 9 "${LARGS[@]}" \
    > gpurun_out/ab/${TAG}_$sh.log 2>&1 || exit $?
  grep -v "^\[" gpurun_out/ab/${TAG}_$sh.log | grep -v "^{" | tail -8
done
