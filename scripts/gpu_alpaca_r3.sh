#!/bin/bash
# Alpaca SFT at Alpaca-shaped lengths (~125 tokens per example, capped at model_max_length 512),
# NB4's batch (mbs 4 x GA 8) on one MI355X:
#   1. OPT-125m, the reference's DS config (ZeRO-3 + offload_param: cpu)  -> opt125m_zero3_offload.log
#   2. OPT-125m, the same data with ZeRO-2                                 -> opt125m_zero2.log
#   3. LLaMA-7B, ZeRO-2 bf16                                               -> llama7b_zero2.log
#   4. LLaMA-7B, ZeRO-2 bf16, mbs 32 x GA 1 (same 32 samples / step), length-grouped -> llama7b_zero2_mbs32.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r3_alpaca2
mkdir -p $O
R=recipes/4_training_alpaca_deepspeed
export HSA_ENABLE_IPC_MODE_LEGACY=0
COMMON="--data_path $O/alpaca.json --synthetic_examples 8192 --bf16 True --num_train_epochs 1 --model_max_length 512 \
 --learning_rate 2e-5 --warmup_ratio 0.03 --save_steps 100000 --tf32 False --report_to none --logging_steps 5 \
 --per_device_train_batch_size 4 --gradient_accumulation_steps 8"
run() {  # name, seconds, args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python -u $R/train.py $COMMON "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc: $(grep -o "'train_input_tokens_per_second'[^}]*" $O/$name.log | tail -1)"
  return $rc
}
run opt125m_zero3_offload 400 --model_name_or_path facebook/opt-125m --output_dir /tmp/a1 --max_steps 60 \
  --deepspeed $R/configs/default_offload_opt_param.json || exit 1
run opt125m_zero2 400 --model_name_or_path facebook/opt-125m --output_dir /tmp/a2 --max_steps 60 \
  --deepspeed $R/configs/zero2_bf16.json || exit 1
run llama7b_zero2 600 --model_name_or_path llama-7b --output_dir /tmp/a3 --max_steps 60 \
  --deepspeed $R/configs/zero2_bf16.json || exit 1
# the same 32 samples per optimizer step as ONE micro-batch (288 GB of HBM holds it), length-grouped
run llama7b_zero2_mbs32 600 --model_name_or_path llama-7b --output_dir /tmp/a4 --max_steps 60 \
  --deepspeed $R/configs/zero2_bf16.json --per_device_train_batch_size 32 --gradient_accumulation_steps 1 \
  --group_by_length True || exit 1
# the same without length grouping (padding to the longest of 32 random examples)
run llama7b_zero2_mbs32_nogroup 600 --model_name_or_path llama-7b --output_dir /tmp/a5 --max_steps 60 \
  --deepspeed $R/configs/zero2_bf16.json --per_device_train_batch_size 32 --gradient_accumulation_steps 1 || exit 1
# NB4's mbs 4 x GA 8 with length grouping
run llama7b_zero2_grouped 600 --model_name_or_path llama-7b --output_dir /tmp/a6 --max_steps 60 \
  --deepspeed $R/configs/zero2_bf16.json --group_by_length True || exit 1
