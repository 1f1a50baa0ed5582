#!/bin/bash
# One GPU session: kernel numerics tests, then the 1-GPU bench, then a rocprofv3 kernel profile.
# Stops at the first step that faults / aborts / times out (exit status not in {0,1}).
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
  tail -n 30 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
TESTS=${TESTS:-tests/test_kernels_gpu.py}
step pytest_gpu 900 python -m pytest $TESTS -q -m gpu
step bench 600 python bench.py --steps ${STEPS:-10} --warmup ${WARMUP:-3} ${BENCH_ARGS:-}
if [ "${PROFILE:-1}" = "1" ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 2 ${BENCH_ARGS:-}
fi
echo DONE
