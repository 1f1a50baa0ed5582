#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "linear_fwd" -m gpu > gpurun_out/pytest_lin.log 2>&1 || { tail -30 gpurun_out/pytest_lin.log; exit 1; }
tail -2 gpurun_out/pytest_lin.log
timeout -k 10 300 python -u benchmarks/bench_linear.py > gpurun_out/bench_linear.log 2>&1 || { tail -20 gpurun_out/bench_linear.log; exit 1; }
cat gpurun_out/bench_linear.log
