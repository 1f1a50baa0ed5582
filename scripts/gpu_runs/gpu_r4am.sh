#!/bin/bash
# Round 4: per-collective stats moved to two extra steps after the timed ones — 1-GPU bench (JSON
# still carries phase_ms / comm) and the per-rank prediction re-measured.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4am
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 1 "$R/$O/$name.log" | cut -c1-200
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step bench 300 python bench.py --steps 20 --warmup 5
step predict 900 python -u benchmarks/predict_scaling.py --merge-json profiles/r4_predict_final/predicted.json \
  --only n1_dp tp2pp2_stage0 tp2pp2_stage1 tp2pp2_stage1_even gpt3_tp4_stage0 gpt3_tp4_stage1 --out $O/predict
grep "zbh2\|tp1pp1dp1 " $O/predict/predicted.md | cut -c1-200
echo DONE
