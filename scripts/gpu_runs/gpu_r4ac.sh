#!/bin/bash
# Round 4: two-rank one-GPU Gloo rehearsal of tp2 + SP after staging the Gloo ring exchange of
# CUDA tensors through host memory; then tp2pp2 (N = 4, zbh2) with four ranks on the GPU.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4ac
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 SMDT_BENCH_BACKEND=gloo SMDT_BENCH_DUMP_AFTER=60
RUN2="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613"
RUN4="python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29614"
timeout -k 10 150 $RUN2 bench.py --gpus 2 --tp 2 --pp 1 --steps 3 --warmup 2 --tunableop 0 --seqs-per-gpu 16 > $O/tp2_sp.log 2>&1
rc=$?; echo "tp2_sp rc=$rc"; grep '^{' $O/tp2_sp.log | cut -c1-400
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 $RUN4 bench.py --gpus 4 --tp 2 --pp 2 --steps 2 --warmup 1 --tunableop 0 --seqs-per-gpu 8 > $O/tp2pp2_zbh2.log 2>&1
echo "tp2pp2_zbh2 rc=$?"; grep '^{' $O/tp2pp2_zbh2.log | cut -c1-400
echo DONE
