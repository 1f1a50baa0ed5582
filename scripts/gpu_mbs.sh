#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/mbs
for spg in 32 64; do
  timeout -k 10 400 python -u bench.py --steps 8 --warmup 3 --seqs-per-gpu $spg > gpurun_out/mbs/spg$spg.log 2>&1 || { tail -20 gpurun_out/mbs/spg$spg.log; exit 1; }
  tail -1 gpurun_out/mbs/spg$spg.log | cut -c1-200
done
timeout -k 10 400 python -u bench.py --steps 8 --warmup 3 --seqs-per-gpu 64 --micro-batch-size 32 > gpurun_out/mbs/spg64_mbs32.log 2>&1 || { tail -20 gpurun_out/mbs/spg64_mbs32.log; exit 1; }
tail -1 gpurun_out/mbs/spg64_mbs32.log | cut -c1-200
