#!/bin/bash
# Full GPU test suite + the default 1-GPU bench, as the round driver runs them.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/final
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/final/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/final/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/final/pytest_gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/final/bench.log 2>&1 || { tail -20 gpurun_out/final/bench.log; exit 1; }
tail -1 gpurun_out/final/bench.log | cut -c1-220
