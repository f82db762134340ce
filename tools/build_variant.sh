#!/bin/bash
# Build a compiler-flag variant of libfa2amd.so for A/B in one process:
#   tools/build_variant.sh <name> "<extra hipcc flags>"  ->  cuda-flash-attention_amd/variants/<name>/libfa2amd.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
N=$1; shift
make -s -j8 -C "$ROOT/cuda-flash-attention_amd" lib BUILD="$ROOT/cuda-flash-attention_amd/variants/$N/build" \
     LIBDIR="$ROOT/cuda-flash-attention_amd/variants/$N" EXTRA="$*"
rm -rf "$ROOT/cuda-flash-attention_amd/variants/$N/build"
