# Sub-batch interleave (SMDT_SP_SUBBATCH=2) on one MI355X: its cost on the emulated N = 8 stage
# rank (loopback exchanges are in-line copies, so only the cost side is visible: half-size
# attention / norm launches, twice the launches), interleaved with the default, eager and graphed;
# then the real 4-process tp2pp2 path over Gloo with the interleave on.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/${OUT:-r5_subbatch}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
ST="--emulate-tp 2 --micro-batch-size 32 --grad-accum 8 --steps 6 --warmup 2"
for i in 1 2; do
  run s1_def_$i 400 python bench.py --num-layers 11 --emulate-last-stage $ST
  SMDT_SP_SUBBATCH=2 run s1_sub_$i 400 python bench.py --num-layers 11 --emulate-last-stage $ST
done
run s0_def 400 python bench.py --num-layers 13 --emulate-first-stage $ST
SMDT_SP_SUBBATCH=2 run s0_sub 400 python bench.py --num-layers 13 --emulate-first-stage $ST
run s1_def_graph 400 python bench.py --num-layers 11 --emulate-last-stage $ST --graph 1
SMDT_SP_SUBBATCH=2 run s1_sub_graph 400 python bench.py --num-layers 11 --emulate-last-stage $ST --graph 1
export SMDT_BENCH_BACKEND=gloo SMDT_SP_SUBBATCH=2
run rehearse_tp2pp2 420 python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --master-port 29534 --nproc-per-node 4 bench.py --steps 2 --warmup 1 --seqs-per-gpu 8 --micro-batch-size 4 --tunableop 0 --gpus 4 --tp 2 --pp 2 --pp-schedule zbh2
echo DONE
