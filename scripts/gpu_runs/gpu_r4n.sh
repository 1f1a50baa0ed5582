#!/bin/bash
# Round 4: elementwise HBM rates (benchmarks/bench_elementwise.py) and the bench, A/B of the flat
# streaming bias-GeLU kernels (SMDT_BA_FLAT=1) against the row-slice form; bias-GeLU GPU tests
# under the flat form.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4n
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 2 "$R/$O/$name.log" | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
SMDT_BA_FLAT=1 step tests_flat 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "bias_gelu or swiglu or mlp"
step ew_rows 120 python benchmarks/bench_elementwise.py
SMDT_BA_FLAT=1 step ew_flat 120 python benchmarks/bench_elementwise.py
step ew_rows2 120 python benchmarks/bench_elementwise.py
SMDT_BA_FLAT=1 step ew_flat2 120 python benchmarks/bench_elementwise.py
step bench_rows 300 python bench.py --steps 20 --warmup 5
SMDT_BA_FLAT=1 step bench_flat 300 python bench.py --steps 20 --warmup 5
echo DONE
