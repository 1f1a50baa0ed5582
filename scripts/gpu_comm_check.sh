#!/bin/bash
# Comm engines (xGMI collectives incl. auto-mode tuning, TP-pair relay) + a 1-GPU bench sanity run.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_relay.py tests/test_xgmi.py -m gpu > gpurun_out/pytest_comm.log 2>&1 || { tail -40 gpurun_out/pytest_comm.log; exit 1; }
tail -2 gpurun_out/pytest_comm.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
