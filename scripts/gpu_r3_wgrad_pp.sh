#!/bin/bash
# A/B of the grouped wgrad kernel: lockstep 8 waves vs ping-pong wave groups (SMDT_WGRAD_PP=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r3_wgrad_pp
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
SMDT_WGRAD_PP=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_parallel_gpu.py tests/test_kernels_gpu.py -k wgrad > $O/pytest_pp.log 2>&1 || { tail -30 $O/pytest_pp.log; exit 1; }
tail -1 $O/pytest_pp.log
for v in 0 1 0 1; do
  SMDT_WGRAD_PP=$v timeout -k 10 200 python -u benchmarks/bench_wgrad.py grouped 4 > $O/grouped_$v.log 2>&1 || { tail -20 $O/grouped_$v.log; exit 1; }
  echo "pp$v: $(tail -1 $O/grouped_$v.log)"
done
for v in 1 0 1; do
  SMDT_WGRAD_PP=$v timeout -k 10 300 python -u bench.py > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  echo "bench pp$v: $(tail -1 $O/bench_$v.log | cut -c1-160)"
done
