#!/bin/bash
# Timing-only ablation builds of the hand-scheduled loops (results invalid, never the product):
#   tools/abl_build.sh name:kernel:abl1,abl2 ...   (kernel: fwd | dq | dkdv; abl names: gen/asmgen.py ABL)
#   -> cuda-flash-attention_amd/abl/<name>/libfa2amd.so
# The kernel sources are copied to abl/<name>/kernels, the generator writes its ablated .inc
# into the copy, and the library is built from the copy (Makefile KDIR); the product source
# tree holds no switch for it.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
P="$ROOT/cuda-flash-attention_amd"
for spec in "$@"; do
  N=${spec%%:*}; rest=${spec#*:}; K=${rest%%:*}; A=${rest#*:}
  D="$P/abl/$N"
  rm -rf "$D" && mkdir -p "$D"
  cp -r "$P/kernels" "$D/kernels"
  case $K in
    fwd)  G=gen_fwd_hs.py;   I=fa2_fwd_hs.inc ;;
    dq)   G=gen_bwd_dq.py;   I=fa2_bwd_dq_hs.inc ;;
    dkdv) G=gen_bwd_dkdv.py; I=fa2_bwd_dkdv_hs.inc ;;
    *) echo "kernel: fwd | dq | dkdv"; exit 2 ;;
  esac
  python3 "$P/gen/$G" --abl "$A" --out "$D/kernels/$I" > /dev/null
  make -s -j8 -C "$P" lib KDIR="$D/kernels" BUILD="$D/build" LIBDIR="$D"
  rm -rf "$D/build" "$D/kernels"
  echo "built $N ($K: $A)"
done
