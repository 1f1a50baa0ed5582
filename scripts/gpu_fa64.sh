#!/bin/bash
# 64-queries-per-wave forward (fwd64_kernel): correctness, then A/B against fwd_kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r3_fa64
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k flash --timeout 120 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 0 1 2; do
  for p in 0.1 0.0; do
    SMDT_FA_FWD64=$v timeout -k 10 120 python benchmarks/bench_attention.py --b 32 --dropout $p --sdpa 0 > $O/attn_v${v}_p${p}.json 2>&1 || exit 1
    echo "fwd64=$v p=$p $(tail -1 $O/attn_v${v}_p${p}.json)"
  done
done
