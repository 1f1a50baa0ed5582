#!/bin/bash
# LLaMA-7B ZeRO-2 SFT step anatomy: NB4's mbs 4 x GA 8 vs mbs 32 x GA 1 (same 32 samples per
# optimizer step), length-grouped batches, and a rocprofv3 kernel summary of the mbs 32 run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r3_alpaca_prof2
mkdir -p $O
export TMPDIR=/tmp
R=recipes/4_training_alpaca_deepspeed
export HSA_ENABLE_IPC_MODE_LEGACY=0
COMMON="--data_path $O/alpaca.json --synthetic_examples 4096 --bf16 True --num_train_epochs 1 --model_max_length 512 \
 --learning_rate 2e-5 --warmup_ratio 0.03 --save_steps 100000 --tf32 False --report_to none --logging_steps 2 \
 --model_name_or_path llama-7b --deepspeed $R/configs/zero2_bf16.json --group_by_length True"
for cfg in "32 1"; do
  set -- $cfg
  timeout -k 10 600 python -u $R/train.py --output_dir /tmp/a_$1 --max_steps 6 --per_device_train_batch_size $1 \
    --gradient_accumulation_steps $2 $COMMON > $O/llama_mbs$1.log 2>&1 || { tail -20 $O/llama_mbs$1.log; exit 1; }
  grep -o "'train_input_tokens_per_second'[^}]*" $O/llama_mbs$1.log | tail -1
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python -u $R/train.py --output_dir /tmp/a_p --max_steps 3 --per_device_train_batch_size 32 \
  --gradient_accumulation_steps 1 $COMMON > $O/llama_prof.log 2>&1 || { tail -20 $O/llama_prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
head -25 "$f" | cut -d, -f1-4 > $O/kernel_stats_top.txt
cat $O/kernel_stats_top.txt
