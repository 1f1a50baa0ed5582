#!/bin/bash
# Round 4: emulated ring exchanges on the loopback side stream (as the real exchange runs beside
# the chunk GEMM): GPU tests, then the tp2pp2 stage ranks A/B (SMDT_LOOPBACK_ASYNC) and the
# refreshed prediction.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4af
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 2 "$R/$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_parallel_gpu.py tests/test_xgmi.py
N8="--emulate-tp 2 --micro-batch-size 32 --grad-accum 8 --steps 6 --warmup 3"
step stage1_async 300 python bench.py $N8 --num-layers 11 --emulate-last-stage
SMDT_LOOPBACK_ASYNC=0 step stage1_inline 300 python bench.py $N8 --num-layers 11 --emulate-last-stage
step predict 800 python -u benchmarks/predict_scaling.py --merge-json profiles/r4_predict_slots/predicted.json \
  --only n1_dp tp2pp2_stage0 tp2pp2_stage1 tp2pp2_stage1_even gpt3_tp4_stage0 gpt3_tp4_stage1 --out $O/predict
echo DONE
