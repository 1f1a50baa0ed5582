#!/bin/bash
# CPU launch overhead at small micro-batches (the per-GPU work of the N = 4 / 8 layouts is
# micro-batch 16 at tp2 ~ micro-batch 8 at full width): bench at mbs 8 and 16 (64 seqs / step),
# plus a kernel trace of the mbs 8 step (kernel-busy vs wall = host gaps).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/smallmb
mkdir -p $O
timeout -k 10 300 python -u bench.py --micro-batch-size 8 > $O/bench_mb8.log 2>&1 || { tail -20 $O/bench_mb8.log; exit 1; }
timeout -k 10 300 python -u bench.py --micro-batch-size 16 > $O/bench_mb16.log 2>&1 || { tail -20 $O/bench_mb16.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --micro-batch-size 8 --steps 3 --warmup 2 > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
f=$(ls $O/prof/*/run_kernel_trace.csv $O/prof/run_kernel_trace.csv 2>/dev/null | head -n 1)
python3 scripts/ktrace_steps.py "$f" > $O/last_step_breakdown.txt 2>&1
head -n 3 $O/last_step_breakdown.txt
for f in bench_mb8 bench_mb16; do tail -1 $O/$f.log | cut -c1-190; done
