#!/bin/bash
# A/B of the grouped wgrad kernel: 8 waves (128 x 64 wave tiles) vs 4 waves (SMDT_WGRAD_WAVES=4,
# 128 x 128 wave tiles, one wave per SIMD, interleaved fragment reads / DMA).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r3_wgrad4
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
SMDT_WGRAD_WAVES=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_parallel_gpu.py tests/test_kernels_gpu.py -k wgrad > $O/pytest4.log 2>&1 || { tail -30 $O/pytest4.log; exit 1; }
tail -1 $O/pytest4.log
for v in 8 4 8 4; do
  SMDT_WGRAD_WAVES=$v timeout -k 10 200 python -u benchmarks/bench_wgrad.py grouped 4 > $O/grouped_$v.log 2>&1 || { tail -20 $O/grouped_$v.log; exit 1; }
  echo "waves$v: $(tail -1 $O/grouped_$v.log)"
done
for v in 4 8 4; do
  SMDT_WGRAD_WAVES=$v timeout -k 10 300 python -u bench.py > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  echo "bench waves$v: $(tail -1 $O/bench_$v.log | cut -c1-160)"
done
