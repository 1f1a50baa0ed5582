#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/ab
for t in 1 0 1; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --tunableop $t > gpurun_out/ab/t$t.log 2>&1 || { tail -20 gpurun_out/ab/t$t.log; exit 1; }
  echo "tunableop=$t $(tail -1 gpurun_out/ab/t$t.log | cut -c1-150)"
done
