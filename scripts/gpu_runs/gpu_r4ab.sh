#!/bin/bash
# Round 4: where the two-rank one-GPU tp2 + SP Gloo rehearsal stalls (thread stacks every 40 s),
# then the same with the TP-pair relay engine off.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4ab
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 SMDT_BENCH_BACKEND=gloo SMDT_BENCH_DUMP_AFTER=40
RUN="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612"
timeout -k 10 130 $RUN bench.py --gpus 2 --tp 2 --pp 1 --steps 3 --warmup 2 --tunableop 0 --seqs-per-gpu 16 > $O/tp2_sp.log 2>&1
echo "tp2_sp rc=$?"
SMDT_TP_RELAY=0 timeout -k 10 130 $RUN bench.py --gpus 2 --tp 2 --pp 1 --steps 3 --warmup 2 --tunableop 0 --seqs-per-gpu 16 > $O/tp2_sp_norelay.log 2>&1
echo "tp2_sp_norelay rc=$?"
grep '^{' $O/tp2_sp_norelay.log | cut -c1-300
echo DONE
