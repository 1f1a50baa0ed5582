#!/bin/bash
# Round 4: kernel traces of the two emulated N = 8 pipeline-stage ranks (tp2 + SP, split backward
# as under zbh1; the last stage now without the embedding), then the tp2pp2 prediction re-measured.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4q
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 2 "$R/$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
N8="--emulate-tp 2 --micro-batch-size 32 --grad-accum 8 --steps 3 --warmup 2"
cd /tmp
step prof_stage1 400 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_stage1" -o run --output-format csv -- \
  python3 "$R/bench.py" $N8 --num-layers 11 --emulate-last-stage
step prof_stage0 400 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_stage0" -o run --output-format csv -- \
  python3 "$R/bench.py" $N8 --num-layers 13 --emulate-first-stage
cd "$R"
for s in stage1 stage0; do
  f=$(find "$O/prof_$s" -name '*kernel_trace.csv' | head -n 1)
  python scripts/ktrace_steps.py "$f" 45 > "$O/${s}_last_step_breakdown.txt" && head -n 12 "$O/${s}_last_step_breakdown.txt"
  find "$O/prof_$s" -name '*kernel_trace.csv' -delete
done
step predict 700 python -u benchmarks/predict_scaling.py --merge-json profiles/r4_predict_split/predicted.json \
  --only n1_dp tp2pp2_stage0 tp2pp2_stage1 tp2pp2_stage1_even --out $O/predict
echo DONE
