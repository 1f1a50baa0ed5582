# round 6: GPT-3 6.7B tp4 pp2 + SP (BASELINE config 5) prediction with the emulated stages measured
# compute-only AND with the SP exchanges through the paced direct-engine stand-in (whole chunks)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r6_predict3; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u benchmarks/predict_scaling.py --out $O --steps 3 --warmup 2 \
  --only gpt3_tp4_stage0 gpt3_tp4_stage1 gpt3_tp4_stage0_direct gpt3_tp4_stage1_direct gpt3_n1 \
  --merge-json profiles/r6_predict2/predicted.json > $O/run.log 2>&1
rc=$?; tail -n 30 $O/run.log; exit $rc
