# round 6: one-GPU Gloo rehearsals (every rank on ONE MI355X; RCCL refuses two ranks per device)
# of the N = 2 / 4 default layouts (dp + ZeRO-1, overlapped bucket reduce-scatters and parameter
# all-gathers) and of the N = 8 pairs with the round-6 exchange overlap defaults (W fillers).
# A small GPT (4 layers, h 512, vocab 8192) keeps Gloo's host-staged CUDA collectives short:
# the point is that each multi-rank path runs end to end on the real kernels, not its speed.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/${OUT:-r6_rehearse}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 SMDT_BENCH_BACKEND=gloo
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --master-port 29533"
B="bench.py --steps 2 --warmup 1 --seqs-per-gpu 8 --micro-batch-size 4 --tunableop 0 --comm-stats 0 \
 --num-layers 4 --hidden-size 512 --num-attention-heads 8 --vocab-size 8192"
run dp4 170 $TR --nproc-per-node 4 $B --gpus 4 --tp 1 --pp 1
run dp2 170 $TR --nproc-per-node 2 $B --gpus 2 --tp 1 --pp 1
run tp2pp2_zbh2_fill 170 $TR --nproc-per-node 4 $B --gpus 4 --tp 2 --pp 2 --pp-schedule zbh2
echo DONE
