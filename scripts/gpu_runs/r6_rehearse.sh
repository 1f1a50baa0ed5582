# round 6: one-GPU Gloo rehearsals of the N = 2 / 4 default layouts (dp + ZeRO-1) and the N = 8
# pairs with the round-6 exchange overlap defaults (W fillers), every rank on ONE MI355X
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/${OUT:-r6_rehearse}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 SMDT_BENCH_BACKEND=gloo
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --master-port 29533"
B="bench.py --steps 2 --warmup 1 --seqs-per-gpu 8 --micro-batch-size 4 --tunableop 0 --comm-stats 0"
run wfill_test 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_parallel_gpu.py -k "w_fillers or fused_mlp_waits"
run dp4_sync 400 $TR --nproc-per-node 4 $B --gpus 4 --tp 1 --pp 1 --overlap-grad-reduce 0
run dp2 400 $TR --nproc-per-node 2 $B --gpus 2 --tp 1 --pp 1
run tp2pp2_zbh2_fill 400 $TR --nproc-per-node 4 $B --gpus 4 --tp 2 --pp 2 --pp-schedule zbh2
echo DONE
