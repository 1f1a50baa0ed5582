# Round-5 check on one MI355X: new GPU tests, vision emulated-DP8 eager vs graph, N = 8 last-stage
# emulation with / without the vocab-parallel fused CE, and a kernel trace of that stage.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=$R/gpurun_out/${OUT:-r5_check}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-700; [ $rc -eq 0 ] || exit $rc; }
run tests 600 python -u -m pytest -q -x --timeout 120 --timeout-method thread -m gpu tests/test_graph_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py
for i in 1 2; do
  run bench_$i 400 python bench.py --steps 20 --warmup 5
  run bench_ovl_$i 400 python bench.py --steps 20 --warmup 5 --overlap-optimizer 1
done
ST="--steps 6 --warmup 2 --num-layers 11 --emulate-last-stage --emulate-tp 2 --micro-batch-size 32 --grad-accum 8"
run stage1_fused 400 python bench.py $ST
SMDT_LM_HEAD_CE=0 run stage1_unfused 400 python bench.py $ST
run stage1_fused2 400 python bench.py $ST
V="--model resnet50 --size 224 --batch 64 --steps 20 --warmup 5 --emulate-dp 8"
run r50_dp8_eager 500 python benchmarks/bench_vision.py $V --graph 0
run r50_dp8_graph 500 python benchmarks/bench_vision.py $V --graph 1 --miopen-prewarm 0
run swin_dp8_eager 500 python benchmarks/bench_vision.py --model swin_b --size 128 --batch 40 --steps 20 --warmup 5 --emulate-dp 8 --graph 0
run swin_dp8_graph 500 python benchmarks/bench_vision.py --model swin_b --size 128 --batch 40 --steps 20 --warmup 5 --emulate-dp 8 --graph 1 --miopen-prewarm 0
run predict 1100 python benchmarks/predict_scaling.py --out "$O/predict" --only n1_dp tp2pp2_stage0 tp2pp2_stage1 tp2pp2_mb64_stage0 tp2pp2_mb64_stage1
cd /tmp
run prof_stage1 400 rocprofv3 --kernel-trace --stats -d "$O/prof_stage1" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 2 --num-layers 11 --emulate-last-stage --emulate-tp 2 --micro-batch-size 32 --grad-accum 8 --comm-stats 0
cd "$R"
f=$(find $O/prof_stage1 -name '*kernel_trace.csv' | head -n 1)
python scripts/ktrace_steps.py "$f" 40 > $O/stage1_last_step_breakdown.txt 2>&1 || echo "breakdown failed"
find $O -name '*kernel_trace.csv' -delete
echo DONE
