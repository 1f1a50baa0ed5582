#!/bin/bash
# xGMI collectives: loopback + cross-process GPU tests, then the loopback kernel benchmark.
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
  tail -n 15 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_xgmi 240 python -u -m pytest tests/test_xgmi.py -x -v -m gpu --timeout 120 --timeout-method thread
step coll_loopback8 120 python benchmarks/bench_collectives.py --loopback 8 --max-mb 64 --iters 10
step coll_loopback2 120 python benchmarks/bench_collectives.py --loopback 2 --max-mb 64 --iters 10
step pytest_attn 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "flash or dropout" --timeout 120 --timeout-method thread
echo DONE
