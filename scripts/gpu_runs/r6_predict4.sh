# round 6: the N = 8 stage ranks under the paced relay stand-in at 4 x 64 and 16 x 16 micro-batches
# (the replica's 256 sequences split differently), merged into the round-6 prediction
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r6_predict4; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u benchmarks/predict_scaling.py --out $O --steps 6 --warmup 3 \
  --only tp2pp2_mb64_stage0_standin tp2pp2_mb64_stage1_standin tp2pp2_mb16_stage0_standin tp2pp2_mb16_stage1_standin \
  --merge-json profiles/r6_predict3/predicted.json > $O/run.log 2>&1
rc=$?; grep -E "^\[predict\]|MEASURED" $O/run.log | cut -c1-400; exit $rc
