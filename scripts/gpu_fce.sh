#!/bin/bash
# Fused LM-head + CE: GPU tests, bench with / without it, rocprof of the fused default.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_fce 300 python -u -m pytest tests/test_model_gpu.py -x -q -m gpu -k "fused_lm_head" --timeout 120 --timeout-method thread
step bench_fce 300 python bench.py --steps 10 --warmup 3
step bench_nofce 300 python bench.py --steps 10 --warmup 3 --no-fused-ce
step rocprof_fce 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 2
echo DONE
