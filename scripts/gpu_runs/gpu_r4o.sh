#!/bin/bash
# Round 4: bias-GeLU launch shape A/B (row slices x2 / x4, 8 rows of loads in flight per thread)
# with benchmarks/bench_elementwise.py, GPU tests under the non-default shapes, then the bench.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4o
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
SMDT_BA_SLICE_MUL=2 SMDT_BA_KROWS=8 step tests_knobs 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "bias_gelu or swiglu or mlp"
step ew_base 120 python benchmarks/bench_elementwise.py
SMDT_BA_SLICE_MUL=2 step ew_s2 120 python benchmarks/bench_elementwise.py
SMDT_BA_SLICE_MUL=4 step ew_s4 120 python benchmarks/bench_elementwise.py
SMDT_BA_KROWS=8 step ew_k8 120 python benchmarks/bench_elementwise.py
SMDT_BA_SLICE_MUL=2 SMDT_BA_KROWS=8 step ew_s2k8 120 python benchmarks/bench_elementwise.py
SMDT_BA_SLICE_MUL=4 SMDT_BA_KROWS=8 step ew_s4k8 120 python benchmarks/bench_elementwise.py
step ew_base2 120 python benchmarks/bench_elementwise.py
echo DONE
