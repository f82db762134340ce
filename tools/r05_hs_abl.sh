#!/bin/bash
# r05: timing-only ablation builds of the hand-scheduled loops (results invalid):
#   tools/r05_hs_abl.sh name:kernel:abl1,abl2 ...   (kernel: fwd | dq | dkdv)
#   -> cuda-flash-attention_amd/abl/<name>/libfa2amd.so
# Only the kernel's translation units are recompiled (the product objects are copied).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
P="$ROOT/cuda-flash-attention_amd"
for spec in "$@"; do
  N=${spec%%:*}; rest=${spec#*:}; K=${rest%%:*}; A=${rest#*:}
  D="$P/abl/$N"
  mkdir -p "$D/build"
  cp -p "$P"/build/*.o "$D/build/"
  case $K in
    fwd)  G=gen_fwd_hs.py;   M=FA2_HS_INC; rm -f "$D"/build/kernel_fa2_optimized_f16.o "$D"/build/kernel_fa2_optimized_bf16.o ;;
    dq)   G=gen_bwd_dq.py;   M=FA2_DQ_INC; rm -f "$D"/build/f-attn2-backward_f16.o "$D"/build/f-attn2-backward_bf16.o ;;
    dkdv) G=gen_bwd_dkdv.py; M=FA2_DK_INC; rm -f "$D"/build/f-attn2-backward_f16.o "$D"/build/f-attn2-backward_bf16.o ;;
  esac
  python3 "$P/gen/$G" --abl "$A" --out "$D/abl.inc" > /dev/null
  make -s -j8 -C "$P" lib BUILD="$D/build" LIBDIR="$D" EXTRA="-D$M=\\\"$D/abl.inc\\\""
  rm -rf "$D/build"
  echo "built $N ($K: $A)"
done
