#!/bin/bash
# A/B of the grouped wgrad kernel: v_mfma_f32_16x16x32 (default) vs 32x32x16 (SMDT_WGRAD_MFMA=32).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r3_wgrad16
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_parallel_gpu.py tests/test_kernels_gpu.py -k wgrad > $O/pytest16.log 2>&1; grep -E "FAILED|passed|failed" $O/pytest16.log
tail -1 $O/pytest16.log
for v in 16 32; do
  SMDT_WGRAD_MFMA=$v timeout -k 10 200 python -u benchmarks/bench_wgrad.py grouped 4 > $O/grouped_$v.log 2>&1 || { tail -20 $O/grouped_$v.log; exit 1; }
  echo "mfma$v: $(tail -1 $O/grouped_$v.log)"
done
for v in 16 32 16; do
  SMDT_WGRAD_MFMA=$v timeout -k 10 300 python -u bench.py > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  echo "bench mfma$v: $(tail -1 $O/bench_$v.log | cut -c1-160)"
done
timeout -k 10 800 python -u benchmarks/predict_scaling.py --out gpurun_out/r3_predict2 > gpurun_out/r3_predict2.log 2>&1 || { tail -20 gpurun_out/r3_predict2.log; exit 1; }
tail -9 gpurun_out/r3_predict2.log
