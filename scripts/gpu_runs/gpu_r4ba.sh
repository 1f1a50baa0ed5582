#!/bin/bash
# Round 4: CE backward load / store forms (SMDT_CE_BWD_VAR 0 nt/nt, 1 nt load + plain store,
# 2 plain / plain) — CE GPU tests under each, elementwise rates interleaved.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4ba
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 1 "$R/$O/$name.log" | cut -c1-420
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for v in 1 2; do
  export SMDT_CE_BWD_VAR=$v; step tests_$v 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "cross or ce_"
done
for r in a b; do
  for v in 0 1 2; do
    export SMDT_CE_BWD_VAR=$v; step ew_${v}_$r 200 python benchmarks/bench_elementwise.py
  done
done
echo DONE
