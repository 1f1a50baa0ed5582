#!/bin/bash
# Round 4: SFT GEMM rates vs packed token count (padding to 256 / 512?) and the full per-rank
# prediction refresh (tp2pp2 stages with the gather slots, GPT-3 TP4 stages, the last stage
# without its embedding).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4s
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
step sft_gemm 200 python benchmarks/bench_sft_gemm_pad.py
step predict 1000 python -u benchmarks/predict_scaling.py --merge-json profiles/r4_predict_zbh2/predicted.json \
  --only n1_dp tp2pp2_stage0 tp2pp2_stage1 tp2pp2_stage1_even gpt3_tp4_stage0 gpt3_tp4_stage1 --out $O/predict
echo DONE
