#!/bin/bash
# Round 4: per-call durations of the bias-epilogue GEMM in the 1-GPU bench step.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4y
mkdir -p "$R/$O"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/$O/prof" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 3 --warmup 3 > "$R/$O/prof.log" 2>&1 || exit $?
cd "$R"
f=$(find "$O/prof" -name '*kernel_trace.csv' | head -n 1)
python scripts/ktrace_calls.py "$f" SK3 > "$O/sk3_calls.txt"
python scripts/ktrace_calls.py "$f" Cijk > "$O/gemm_calls.txt"
find "$O/prof" -name '*kernel_trace.csv' -delete
head -n 30 "$O/sk3_calls.txt"
