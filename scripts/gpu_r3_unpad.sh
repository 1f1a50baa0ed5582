#!/bin/bash
# dK/dV overlapped halves: attention tests + microbench; LLaMA SFT padding-free + W^T cache.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r3_unpad
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=recipes/4_training_alpaca_deepspeed
COMMON="--data_path $O/alpaca.json --synthetic_examples 8192 --bf16 True --num_train_epochs 1 --model_max_length 512 \
 --learning_rate 2e-5 --warmup_ratio 0.03 --save_steps 100000 --tf32 False --report_to none --logging_steps 5 \
 --model_name_or_path llama-7b --deepspeed $R/configs/zero2_bf16.json --max_steps 60"
timeout -k 10 600 python -u $R/train.py $COMMON --output_dir /tmp/b1 --per_device_train_batch_size 4 \
  --gradient_accumulation_steps 8 > $O/llama_mbs4.log 2>&1 || { tail -20 $O/llama_mbs4.log; exit 1; }
echo "mbs4 ga8: $(grep -o "'train_input_tokens_per_second'[^}]*" $O/llama_mbs4.log | tail -1)"
timeout -k 10 600 python -u $R/train.py $COMMON --output_dir /tmp/b2 --per_device_train_batch_size 32 \
  --gradient_accumulation_steps 1 > $O/llama_mbs32.log 2>&1 || { tail -20 $O/llama_mbs32.log; exit 1; }
echo "mbs32 ga1: $(grep -o "'train_input_tokens_per_second'[^}]*" $O/llama_mbs32.log | tail -1)"
SMDT_SFT_UNPAD=0 timeout -k 10 600 python -u $R/train.py $COMMON --output_dir /tmp/b3 --per_device_train_batch_size 32 \
  --gradient_accumulation_steps 1 > $O/llama_mbs32_padded.log 2>&1 || { tail -20 $O/llama_mbs32_padded.log; exit 1; }
echo "mbs32 ga1 padded: $(grep -o "'train_input_tokens_per_second'[^}]*" $O/llama_mbs32_padded.log | tail -1)"
