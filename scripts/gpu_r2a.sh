#!/bin/bash
# Round-2 GPU session A: full GPU test suite, default bench, micro-batch-16 bench (per-GPU shape of
# the tp2pp2 layout's micro-batches), each step under its own time limit; stops at the first
# step that faults / aborts / times out.
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
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 900 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread
step bench 300 python bench.py --steps 10 --warmup 3
step bench_mbs16 300 python bench.py --steps 5 --warmup 2 --micro-batch-size 16 --grad-accum 2
echo DONE
