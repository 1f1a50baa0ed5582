#!/bin/bash
# hipBLASLt epilogue MLP: numerics test, microbenchmark, bench A/B (SMDT_MLP_EPILOGUE 0 / 1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r3_mlp_ep
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gelu_mlp or bias_gelu" --timeout 120 \
  --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
SMDT_LINEAR_EP_LOG=1 timeout -k 10 200 python benchmarks/bench_mlp_epilogue.py > $O/micro.log 2>&1 || { tail -20 $O/micro.log; exit 1; }
grep -v summary $O/micro.log
for v in 0 1; do
  SMDT_MLP_EPILOGUE=$v timeout -k 10 300 python bench.py --steps 10 --warmup 4 > $O/bench_ep$v.log 2>&1 || { tail -20 $O/bench_ep$v.log; exit 1; }
  echo "ep=$v $(grep '^{' $O/bench_ep$v.log | tail -1 | cut -c1-200)"
done
