# round 6: same-call A/B of the round-5 tree (worktree _ab_r5 at 75c7438, its own build) against
# this tree on the emulated stage ranks and the GPT-3 TP4 stage, then the full GPU suite, smoke
# and the N = 1 bench of this tree
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/${OUT:-r6_ab}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
ST="--emulate-tp 2 --micro-batch-size 32 --grad-accum 8 --steps 6 --warmup 3 --num-layers 13 --emulate-first-stage"
G="--emulate-tp 4 --hidden-size 4096 --num-attention-heads 32 --seq-length 2048 --micro-batch-size 4 --grad-accum 8 --tunableop 0 --steps 3 --warmup 2 --num-layers 16 --emulate-first-stage"
export SMDT_W_FILL=0 SMDT_RING_GEMM_TN=0
for i in 1 2; do
  ( cd $R/_ab_r5 && run s0_r5_$i 400 python bench.py $ST ) || exit 1
  run s0_r6_$i 400 python bench.py $ST
done
( cd $R/_ab_r5 && run g0_r5 500 python bench.py $G ) || exit 1
run g0_r6 500 python bench.py $G
SMDT_FUSED_BIAS_GELU=0 run g0_r6_nofusedmlp 500 python bench.py $G
unset SMDT_W_FILL SMDT_RING_GEMM_TN
run pytest_gpu 1000 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests
run smoke 180 python __graft_entry__.py smoke
run bench 400 python bench.py --steps 20 --warmup 5
echo DONE
