#!/bin/bash
# Round 4: batch-per-thread Adam (now the only form) — optimizer / kernel GPU tests, Adam rate;
# LayerNorm forward without the 2048-block grid cap (SMDT_LN_FWD_UNCAP A/B); bench.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4at
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 1 "$R/$O/$name.log" | cut -c1-230
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step tests 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests
step adam 120 python benchmarks/bench_adam.py
step ew_cap 120 python benchmarks/bench_elementwise.py
SMDT_LN_FWD_UNCAP=1 step ew_uncap 120 python benchmarks/bench_elementwise.py
step ew_cap2 120 python benchmarks/bench_elementwise.py
SMDT_LN_FWD_UNCAP=1 step ew_uncap2 120 python benchmarks/bench_elementwise.py
step bench 300 python bench.py --steps 20 --warmup 5
SMDT_LN_FWD_UNCAP=1 step bench_uncap 300 python bench.py --steps 20 --warmup 5
echo DONE
