#!/bin/bash
# Per-kernel VGPRs / spills / LDS / occupancy of one kernel source (hipcc remarks), as a table.
# usage: tools/resource_usage.sh <file.cu> [grep-pattern] [extra hipcc flags...]
f=$1; pat=${2:-.}; shift 2 2>/dev/null
ROOT=$(cd "$(dirname "$0")/.." && pwd)
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -mllvm -amdgpu-mfma-vgpr-form=1 -fno-slp-vectorize \
  -I$ROOT/include -I$ROOT/cuda-flash-attention_amd/kernels "$@" -x hip -c "$f" -o /tmp/ru_$$.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | sed -n 's/.*remark: *//p' | awk '
  /Function Name:/ {if (n) print line; n=1; split($0,a,": "); line=a[2]; sub(/ \[.*/,"",line); next}
  /VGPRs:|VGPRs Spill:|LDS Size|Occupancy/ {v=$0; sub(/ \[-Rpass.*/,"",v); gsub(/ +/," ",v); line=line " | " v}
  END {if (n) print line}' | c++filt | grep -E "$pat"
rm -f /tmp/ru_$$.o
