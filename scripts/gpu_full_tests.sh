#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu_all.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_all.log
exit $rc
