#!/bin/bash
# r05: timing-only ablation builds of the hand-scheduled forward loop (results invalid):
#   tools/r05_hs_abl.sh name:abl1,abl2 ...  ->  cuda-flash-attention_amd/abl/<name>/libfa2amd.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
for spec in "$@"; do
  N=${spec%%:*}; A=${spec#*:}
  D="$ROOT/cuda-flash-attention_amd/abl/$N"
  mkdir -p "$D"
  python3 "$ROOT/cuda-flash-attention_amd/gen/gen_fwd_hs.py" --abl "$A" --out "$D/fa2_fwd_hs.inc" > /dev/null
  make -s -j8 -C "$ROOT/cuda-flash-attention_amd" lib BUILD="$D/build" LIBDIR="$D" \
       EXTRA="-DFA2_HS_INC=\\\"$D/fa2_fwd_hs.inc\\\""
  rm -rf "$D/build"
  echo "built $N ($A)"
done
