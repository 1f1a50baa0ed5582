#!/bin/bash
# Round 4: the per-rank prediction re-measured on the final tree (tp2pp2 stage ranks, GPT-3 TP4
# stage ranks, N = 1).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/${R4AG_OUT:-r4ag}
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u benchmarks/predict_scaling.py --merge-json profiles/r4_predict_final2/predicted.json \
  --only n1_dp tp2pp2_stage0 tp2pp2_stage1 tp2pp2_stage1_even gpt3_tp4_stage0 gpt3_tp4_stage1 --out $O/predict > $O/predict.log 2>&1
echo "predict rc=$?"
grep "zbh2\|gpt3\|tp1pp1dp1 " $O/predict/predicted.md | cut -c1-220
