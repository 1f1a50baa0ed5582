#!/bin/bash
# Per-rank compute of GPT-3 6.7B at TP4 PP2 (BASELINE config #5) on ONE MI355X: one pipeline
# stage (16 of 32 layers) at quarter width (8 of 32 heads, ffn 16384 / 4, vocab 50304 / 4),
# seq 2048, 32 sequences per step as 8 micro-batches of 4; plus the whole 6.7B model on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r3_gpt3
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
A="--hidden-size 4096 --seq-length 2048 --tunableop 0 --steps 4 --warmup 2"
timeout -k 10 500 python -u bench.py $A --num-layers 16 --num-attention-heads 8 --kv-channels 128 --ffn-hidden-size 4096 \
  --vocab-size 12576 --seqs-per-gpu 32 --micro-batch-size 4 --grad-accum 8 > $O/rank_stage1.log 2>&1 || { tail -20 $O/rank_stage1.log; exit 1; }
echo "rank (stage 1: 16 layers + head): $(grep '^{' $O/rank_stage1.log | tail -1 | cut -c1-220)"
timeout -k 10 500 python -u bench.py $A --num-layers 16 --num-attention-heads 8 --kv-channels 128 --ffn-hidden-size 4096 \
  --vocab-size 12576 --seqs-per-gpu 32 --micro-batch-size 4 --grad-accum 8 --emulate-first-stage > $O/rank_stage0.log 2>&1 || { tail -20 $O/rank_stage0.log; exit 1; }
echo "rank (stage 0: 16 layers + embedding): $(grep '^{' $O/rank_stage0.log | tail -1 | cut -c1-220)"
timeout -k 10 600 python -u bench.py $A --num-layers 32 --num-attention-heads 32 --vocab-size 50257 --seqs-per-gpu 4 \
  --micro-batch-size 4 --grad-accum 1 > $O/n1_full.log 2>&1 || { tail -20 $O/n1_full.log; exit 1; }
echo "n1 full 6.7B: $(grep '^{' $O/n1_full.log | tail -1 | cut -c1-220)"
