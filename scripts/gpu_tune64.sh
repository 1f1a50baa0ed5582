#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/tune
timeout -k 10 1000 python -u scripts/tune_gemm_shapes.py --out gpurun_out/tune/shapes.csv --tune-ms 30 --iters 3 > gpurun_out/tune/shapes.log 2>&1 || { tail -20 gpurun_out/tune/shapes.log; exit 1; }
tail -3 gpurun_out/tune/shapes.log
