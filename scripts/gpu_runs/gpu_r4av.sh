#!/bin/bash
# Round 4: GPU suite + smoke + elementwise rates + bench on the tree with the 2-D SwiGLU kernels.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4av
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
step pytest_gpu 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests
step smoke 180 python __graft_entry__.py smoke
step ew 150 python benchmarks/bench_elementwise.py
step bench 300 python bench.py --steps 20 --warmup 5
step bench2 300 python bench.py --steps 20 --warmup 5
echo DONE
