#!/bin/bash
# Rehearsal of bench.py's N = 2 / 4 / 8 layouts with every rank on ONE MI355X (Gloo process
# groups: RCCL refuses two ranks on one device). Exercises the DP / ZeRO-1 / TP + SP / PP code
# paths with the real HIP kernels; the numbers are NOT throughput (ranks share one GPU).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 SMDT_BENCH_BACKEND=gloo SMDT_BENCH_DUMP_AFTER=100
O=gpurun_out/r3_rehearse
mkdir -p $O
run() {  # nproc, extra args, log name
  timeout -k 10 170 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 \
    --master-port $((29500 + $1)) bench.py --gpus $1 --steps 2 --warmup 1 --tunableop 0 $2 > $O/$3.log 2>&1 || { tail -30 $O/$3.log; exit 1; }
  echo "$3: $(grep '^{' $O/$3.log | tail -1 | cut -c1-400)"
}
run 4 "--seqs-per-gpu 8" n4_dp4
run 8 "--seqs-per-gpu 8" n8_tp2pp2dp2
