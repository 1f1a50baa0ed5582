#!/bin/bash
# Like-for-like GPT-2 small (NB3 shape: mbs 12 x GA 4) on one MI355X: merged accumulation-window
# wgrad forced on (SMDT_WGRAD_MERGE_ACCUM=1) / off (0) / the schedule's default (off since r3_l4l).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r3_l4l
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in 1 0 default; do
  ( [ $v = default ] || export SMDT_WGRAD_MERGE_ACCUM=$v; exec timeout -k 10 300 python -u bench.py --num-layers 12 --hidden-size 768 --num-attention-heads 12 \
    --seqs-per-gpu 48 --micro-batch-size 12 --grad-accum 4 --steps 10 --warmup 3 ) > $O/gpt2_small_merge$v.log 2>&1 \
    || { tail -20 $O/gpt2_small_merge$v.log; exit 1; }
  echo "merge=$v: $(grep '^{' $O/gpt2_small_merge$v.log | tail -1 | cut -c1-200)"
done
