#!/bin/bash
# Round 4: bias-first tile order spread over the XCDs (every XCD's first tiles are its share of
# the bias tiles) vs the plain problem order (SMDT_WGRAD_BIAS_FIRST=0), same box.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4ao
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 1 "$R/$O/$name.log" | cut -c1-330
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_parallel_gpu.py tests/test_model_gpu.py
step wb_first 200 python benchmarks/bench_wgrad_bias.py --layers 8
SMDT_WGRAD_BIAS_FIRST=0 step wb_plain 200 python benchmarks/bench_wgrad_bias.py --layers 8
step wb_first2 200 python benchmarks/bench_wgrad_bias.py --layers 8
SMDT_WGRAD_BIAS_FIRST=0 step wb_plain2 200 python benchmarks/bench_wgrad_bias.py --layers 8
step bench_first 300 python bench.py --steps 20 --warmup 5
SMDT_WGRAD_BIAS_FIRST=0 step bench_plain 300 python bench.py --steps 20 --warmup 5
step bench_first2 300 python bench.py --steps 20 --warmup 5
SMDT_WGRAD_BIAS_FIRST=0 step bench_plain2 300 python bench.py --steps 20 --warmup 5
echo DONE
