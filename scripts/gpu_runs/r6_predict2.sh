# round 6: predictor stand-in rows re-measured with the filler-stream default (r6_fill3)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/${OUT:-r6_predict2}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u benchmarks/predict_scaling.py --out $O --only n1_dp tp2pp2_stage0_standin tp2pp2_stage1_standin \
  --merge-json profiles/r6_predict/predicted.json > $O/run.log 2>&1
rc=$?; tail -n 30 $O/run.log; echo "rc=$rc"; exit $rc
