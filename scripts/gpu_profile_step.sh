#!/bin/bash
# Kernel-trace profile of the default bench step + per-step breakdown (profiles/<dir>).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof_bench.log 2>&1 || { tail -20 gpurun_out/prof_bench.log; exit 1; }
f=$(ls gpurun_out/prof/*/run_kernel_trace.csv gpurun_out/prof/run_kernel_trace.csv 2>/dev/null | head -n 1)
python3 scripts/ktrace_steps.py "$f" > gpurun_out/last_step_breakdown.txt 2>&1
head -n 30 gpurun_out/last_step_breakdown.txt
