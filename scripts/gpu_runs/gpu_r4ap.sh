#!/bin/bash
# Round 4: bias-GeLU launch shape, more row slices (x8, x16) than the default x4.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4ap
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for v in 4 8 16 4 8 16; do
  SMDT_BA_SLICE_MUL=$v timeout -k 10 120 python benchmarks/bench_elementwise.py >> $O/ew.log 2>&1 || exit $?
done
grep '^{' $O/ew.log | cut -c1-160
