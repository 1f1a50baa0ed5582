#!/bin/bash
# Round 4: bias-first tile order in the grouped wgrad (bias column-sum tiles grouped into the first
# round of a launch) — wgrad GPU tests, the bias-fusion cost microbench (no bias vs the step's
# QKV / fc1 biases vs all biases, same launch shapes), and the bench.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4an
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 1 "$R/$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_parallel_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py
step wgrad_bias 200 python benchmarks/bench_wgrad_bias.py --layers 8
step wgrad_bias2 200 python benchmarks/bench_wgrad_bias.py --layers 8
step bench 300 python bench.py --steps 20 --warmup 5
step bench2 300 python bench.py --steps 20 --warmup 5
echo DONE
