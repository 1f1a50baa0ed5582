# round 6, final tree: full GPU suite, smoke, N = 1 bench twice, a kernel trace of the bench step,
# and the one-GPU Gloo rehearsal of tp2pp2 zbh2 with the filler-stream default
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/${OUT:-r6_final}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
run pytest_gpu 900 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests
run smoke 180 python __graft_entry__.py smoke
run bench 400 python bench.py --steps 20 --warmup 5
run bench_2 400 python bench.py --steps 20 --warmup 5
cd /tmp
run prof 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 3
cd $R
f=$(find $O/prof -name '*kernel_trace.csv' | head -n 1)
python scripts/ktrace_steps.py "$f" 40 > $O/last_step_breakdown.txt && head -n 16 $O/last_step_breakdown.txt
find $O/prof -name '*kernel_trace.csv' -delete
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --master-port 29533"
B="bench.py --steps 2 --warmup 1 --seqs-per-gpu 8 --micro-batch-size 4 --tunableop 0 --comm-stats 0 \
 --num-layers 4 --hidden-size 512 --num-attention-heads 8 --vocab-size 8192"
SMDT_BENCH_BACKEND=gloo run tp2pp2_zbh2_fillstream 170 $TR --nproc-per-node 4 $B --gpus 4 --tp 2 --pp 2 --pp-schedule zbh2
echo DONE
