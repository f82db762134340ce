#!/bin/bash
# GPU box: smoke, then pytest -m gpu (PYTEST_K selects a subset), then optional
# kbench lines (KBENCH="shape|kernels|variants;..."); every GPU step time-limited,
# the script stops at the first crash / abort / timeout.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
fatal() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; fatal $rc && exit $rc
if [ -n "${PYTEST_K}" ]; then KARG=(-k "${PYTEST_K}"); else KARG=(); fi
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider "${KARG[@]}" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log; fatal $rc && exit $rc
IFS=';' read -ra KB <<< "${KBENCH}"
n=0
for spec in "${KB[@]}"; do
  [ -z "$spec" ] && continue
  IFS='|' read -r shape kern vars <<< "$spec"
  args=(--shape "$shape")
  for k in $kern; do args+=(--kernel "$k"); done
  for v in $vars; do args+=(--variant "$v"); done
  n=$((n+1))
  timeout -k 10 300 python tools/kbench.py "${args[@]}" > gpurun_out/kbench_$n.log 2>&1
  rc=$?; echo "kbench $n ($spec) rc=$rc"; grep -v "^\[" gpurun_out/kbench_$n.log | grep -v "^{" | tail -12; fatal $rc && exit $rc
done
exit 0
