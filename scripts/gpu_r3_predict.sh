#!/bin/bash
# GPU suite on the trimmed tree + refreshed per-N scaling prediction (benchmarks/predict_scaling.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_predict3
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 900 python -u benchmarks/predict_scaling.py --out $O > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
tail -9 $O/run.log
