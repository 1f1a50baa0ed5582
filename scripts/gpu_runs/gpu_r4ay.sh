#!/bin/bash
# Round 4: LayerNorm backward block count (512 default vs 1024 / 2048; partial slab grows).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4ay
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for b in 512 1024 2048 256 512 1024 2048; do
  SMDT_LN_BWD_BLOCKS=$b timeout -k 10 200 python benchmarks/bench_elementwise.py > $O/ew_$b.log 2>&1 || exit $?
  echo "$b $(grep -o '"ln_bwd_incl_autograd": {[^}]*}' $O/ew_$b.log)"
done
for b in 512 1024 512 1024; do
  SMDT_LN_BWD_BLOCKS=$b timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_$b.log 2>&1 || exit $?
  echo "bench $b $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$b.log | head -n 1)"
done
