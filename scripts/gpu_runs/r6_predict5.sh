# round 6, final tree: the N = 8 (GPT-2 345M tp2pp2dp2) prediction re-measured in one call —
# N = 1, the compute-only stage ranks and the stage ranks under the paced relay stand-in
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r6_predict5; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1100 python -u benchmarks/predict_scaling.py --out $O --steps 6 --warmup 3 \
  --only n1_dp tp2pp2_stage0 tp2pp2_stage1 tp2pp2_stage0_standin tp2pp2_stage1_standin \
  --merge-json profiles/r6_predict4/predicted.json > $O/run.log 2>&1
rc=$?; grep -E "^\[predict\]|MEASURED|TP exchange relay" $O/run.log | cut -c1-330; exit $rc
