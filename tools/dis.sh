#!/bin/bash
# Device disassembly of one kernel source (gfx950), same flags as the Makefile.
# usage: tools/dis.sh <file.cu> <out.txt> [extra hipcc flags...]
f=$1; out=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -mllvm -amdgpu-mfma-vgpr-form=1 -fno-slp-vectorize \
  -I$ROOT/include -I$ROOT/cuda-flash-attention_amd/kernels "$@" -x hip --cuda-device-only --no-gpu-bundle-output -c "$f" -o /tmp/dis_$$.co &&
/opt/rocm/lib/llvm/bin/llvm-objdump -d --no-show-raw-insn /tmp/dis_$$.co > "$out"
rc=$?; rm -f /tmp/dis_$$.co; exit $rc
