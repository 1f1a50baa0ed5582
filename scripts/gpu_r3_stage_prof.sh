#!/bin/bash
# Kernel-trace profile of the N = 8 per-rank emulation (tp2 pp2 last stage: 11 layers at half width
# + half-vocab LM head, 256 sequences as 8 micro-batches of 32) next to the N = 1 step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_stage_prof
mkdir -p $O
ARGS="--num-layers 11 --num-attention-heads 8 --kv-channels 64 --ffn-hidden-size 2048 --vocab-size 25152 --seqs-per-gpu 256 --micro-batch-size 32 --grad-accum 8"
timeout -k 10 300 python -u bench.py $ARGS --steps 6 --warmup 3 --comm-stats 1 > $O/stage1.log 2>&1 || { tail -20 $O/stage1.log; exit 1; }
tail -1 $O/stage1.log | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py $ARGS --steps 2 --warmup 2 > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
f=$(ls $O/prof/*/run_kernel_trace.csv $O/prof/run_kernel_trace.csv 2>/dev/null | head -n 1)
python3 scripts/ktrace_steps.py "$f" > $O/last_step_breakdown.txt 2>&1
head -n 40 $O/last_step_breakdown.txt
