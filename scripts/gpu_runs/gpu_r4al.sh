#!/bin/bash
# Round 4: host cost of the per-collective stats (--comm-stats, default on): emulated N = 8 stage
# rank and the 1-GPU bench with stats on / off, same box.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4al
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  grep -o '"ms_per_step": [0-9.]*' "$R/$O/$name.log" | tail -n 1
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
N8="--emulate-tp 2 --micro-batch-size 32 --grad-accum 8 --steps 6 --warmup 3"
step stage1_stats 300 python bench.py $N8 --num-layers 11 --emulate-last-stage --comm-stats 1
step stage1_nostats 300 python bench.py $N8 --num-layers 11 --emulate-last-stage --comm-stats 0
step stage1_stats2 300 python bench.py $N8 --num-layers 11 --emulate-last-stage --comm-stats 1
step stage1_nostats2 300 python bench.py $N8 --num-layers 11 --emulate-last-stage --comm-stats 0
step n1_stats 300 python bench.py --steps 20 --warmup 5 --comm-stats 1
step n1_nostats 300 python bench.py --steps 20 --warmup 5 --comm-stats 0
echo DONE
