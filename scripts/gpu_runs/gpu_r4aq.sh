#!/bin/bash
# Round 4: bias-GeLU launch shape sweep around one 8-row batch per thread (slices x16 .. x64,
# 4 / 8 rows in flight), then the bench at the default (x4) and x16.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4aq
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for cfg in "16 8" "32 8" "64 8" "16 4" "32 4" "64 4" "16 8" "32 4"; do
  set -- $cfg
  SMDT_BA_SLICE_MUL=$1 SMDT_BA_KROWS=$2 timeout -k 10 120 python benchmarks/bench_elementwise.py >> $O/ew.log 2>&1 || exit $?
done
grep '^{' $O/ew.log | cut -c1-170
for v in 4 16 4 16; do
  SMDT_BA_SLICE_MUL=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_s$v.log 2>&1 || exit $?
  echo "s$v $(grep -o '"ms_per_step": [0-9.]*' $O/bench_s$v.log | head -n 1)"
done
