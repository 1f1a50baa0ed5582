# round 6: N = 1 bench + the N = 8 stage ranks, compute-only and under the paced relay stand-in
# with the exchange overlap on; predicted.md from them (GPT-3 rows from round 5's measurements)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/${OUT:-r6_predict}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u benchmarks/predict_scaling.py --out $O --only n1_dp tp2pp2_stage0 tp2pp2_stage1 \
  tp2pp2_stage0_standin tp2pp2_stage1_standin --merge-json profiles/r5_predict_final/predicted.json > $O/run.log 2>&1
rc=$?; tail -n 30 $O/run.log; echo "rc=$rc"; exit $rc
