# One-GPU Gloo rehearsals of the N = 2 / 4 default layouts (pure DP + ZeRO-1) on the final tree.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r5_rehearse_dp; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 SMDT_BENCH_BACKEND=gloo
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --master-port 29535"
B="bench.py --steps 2 --warmup 1 --seqs-per-gpu 8 --micro-batch-size 8 --tunableop 0"
run dp2 420 $TR --nproc-per-node 2 $B --gpus 2
run dp4 420 $TR --nproc-per-node 4 $B --gpus 4
echo DONE
