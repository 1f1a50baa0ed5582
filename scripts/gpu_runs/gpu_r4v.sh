#!/bin/bash
# Round 4: kernel trace of the LLaMA-7B NB4 SFT emulated DP8 rank with row-split GEMMs.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4v
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
SF=recipes/4_training_alpaca_deepspeed
COMMON="--data_path $R/$O/alpaca.json --synthetic_examples 4096 --bf16 True --num_train_epochs 1 --model_max_length 512 \
 --learning_rate 2e-5 --warmup_ratio 0.03 --save_steps 100000 --tf32 False --report_to none --logging_steps 4 \
 --model_name_or_path llama-7b --deepspeed $R/$SF/configs/zero2_bf16.json --per_device_train_batch_size 4 --gradient_accumulation_steps 8"
cd /tmp
SMDT_EMULATE_DP=8 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv -- \
  python3 -u "$R/$SF/train.py" $COMMON --max_steps 10 --output_dir /tmp/m2 > "$R/$O/prof.log" 2>&1
rc=$?
echo "prof rc=$rc"
[ $rc -ne 0 ] && exit $rc
cd "$R"
f=$(find "$O/prof" -name '*kernel_trace.csv' | head -n 1)
python scripts/ktrace_steps.py "$f" 40 > "$O/sft_dp8_rank_step_breakdown.txt" && head -n 25 "$O/sft_dp8_rank_step_breakdown.txt"
find "$O/prof" -name '*kernel_trace.csv' -delete
echo DONE
