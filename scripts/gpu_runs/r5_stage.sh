# Emulated N = 8 last-stage rank on one MI355X: fused vs unfused vocab-parallel LM-head CE (kernel
# stats of each), eager vs whole-step HIP graph; the new graph / RNG GPU tests.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=$R/gpurun_out/${OUT:-r5_stage}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
run tests 600 python -u -m pytest -q -x --timeout 150 --timeout-method thread -m gpu tests/test_graph_gpu.py tests/test_kernels_gpu.py -k "graph or rng or vocab_parallel"
ST="--num-layers 11 --emulate-last-stage --emulate-tp 2 --micro-batch-size 32 --grad-accum 8"
run st_eager 400 python bench.py --steps 6 --warmup 2 $ST
run st_graph 400 python bench.py --steps 6 --warmup 2 $ST --graph 1
run st_eager2 400 python bench.py --steps 6 --warmup 2 $ST
run st_graph2 400 python bench.py --steps 6 --warmup 2 $ST --graph 1
cd /tmp
run prof_fused 300 rocprofv3 --kernel-trace --stats -d "$O/prof_fused" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 $ST --comm-stats 0
SMDT_LM_HEAD_CE=0 run prof_unfused 300 rocprofv3 --kernel-trace --stats -d "$O/prof_unfused" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 $ST --comm-stats 0
cd "$R"
for v in fused unfused; do
  f=$(find $O/prof_$v -name '*kernel_trace.csv' | head -n 1)
  python scripts/ktrace_steps.py "$f" 45 > $O/${v}_last_step.txt 2>&1 || echo "breakdown $v failed"
done
find $O -name '*kernel_trace.csv' -delete
echo DONE
