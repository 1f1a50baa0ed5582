#!/bin/bash
# TN-dgrad change: kernel tests, the layout microbenchmark, then the default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/dgrad
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "transpose or dgrad" > gpurun_out/dgrad/pytest.log 2>&1 || { tail -30 gpurun_out/dgrad/pytest.log; exit 1; }
tail -1 gpurun_out/dgrad/pytest.log
timeout -k 10 200 python -u benchmarks/bench_dgrad.py > gpurun_out/dgrad/bench_dgrad.log 2>&1 || { tail -20 gpurun_out/dgrad/bench_dgrad.log; exit 1; }
timeout -k 10 200 python -u benchmarks/bench_dgrad.py --m 16384 > gpurun_out/dgrad/bench_dgrad16k.log 2>&1 || { tail -20 gpurun_out/dgrad/bench_dgrad16k.log; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/dgrad/bench_tn.log 2>&1 || { tail -20 gpurun_out/dgrad/bench_tn.log; exit 1; }
SMDT_DGRAD_TN=0 timeout -k 10 300 python -u bench.py > gpurun_out/dgrad/bench_nn.log 2>&1 || { tail -20 gpurun_out/dgrad/bench_nn.log; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/dgrad/bench_tn2.log 2>&1 || { tail -20 gpurun_out/dgrad/bench_tn2.log; exit 1; }
for f in bench_tn bench_nn bench_tn2; do tail -1 gpurun_out/dgrad/$f.log | cut -c1-200; done
