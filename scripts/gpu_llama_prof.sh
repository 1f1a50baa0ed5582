#!/bin/bash
# LLaMA-7B ZeRO-2 padding-free SFT step anatomy (mbs 32 x GA 1): rocprofv3 kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r3_llama_prof
mkdir -p $O
export TMPDIR=/tmp
R=recipes/4_training_alpaca_deepspeed
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python -u $R/train.py --data_path $O/alpaca.json --synthetic_examples 4096 --bf16 True --num_train_epochs 1 \
  --model_max_length 512 --learning_rate 2e-5 --warmup_ratio 0.03 --save_steps 100000 --tf32 False --report_to none \
  --logging_steps 2 --model_name_or_path llama-7b --deepspeed $R/configs/zero2_bf16.json --output_dir /tmp/p1 \
  --max_steps 8 --per_device_train_batch_size 32 --gradient_accumulation_steps 1 > $O/train.log 2>&1 \
  || { tail -20 $O/train.log; exit 1; }
grep -o "'train_input_tokens_per_second'[^}]*" $O/train.log | tail -1
