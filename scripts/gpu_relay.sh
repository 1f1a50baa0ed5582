#!/bin/bash
# Relay exchange: loopback + cross-process tests, xGMI regression tests, TP tests.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_relay.py tests/test_xgmi.py -m gpu > gpurun_out/pytest_relay.log 2>&1 || { tail -40 gpurun_out/pytest_relay.log; exit 1; }
tail -3 gpurun_out/pytest_relay.log
timeout -k 10 180 python -u benchmarks/bench_collectives.py --loopback 8 --max-mb 64 --region-mb 16 > gpurun_out/relay_loopback8.log 2>&1 || { tail -20 gpurun_out/relay_loopback8.log; exit 1; }
grep pair_exchange gpurun_out/relay_loopback8.log
