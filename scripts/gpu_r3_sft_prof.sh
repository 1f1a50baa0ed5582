#!/bin/bash
# Kernel trace of LLaMA-7B Alpaca SFT at the NB4 config (mbs 4 x GA 8, ZeRO-2, padding-free,
# merged accumulation window): per-step kernel-busy vs wall (launch-bound?) and the top kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3_sft_prof
mkdir -p $O
R=recipes/4_training_alpaca_deepspeed
COMMON="--data_path $O/alpaca.json --synthetic_examples 2048 --bf16 True --num_train_epochs 1 --model_max_length 512 \
 --learning_rate 2e-5 --warmup_ratio 0.03 --save_steps 100000 --tf32 False --report_to none --logging_steps 2 \
 --model_name_or_path llama-7b --deepspeed $R/configs/zero2_bf16.json --max_steps 6 \
 --per_device_train_batch_size 4 --gradient_accumulation_steps 8 --output_dir /tmp/sp"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u $R/train.py $COMMON > $O/train.log 2>&1 || { tail -20 $O/train.log; exit 1; }
f=$(ls $O/prof/*/run_kernel_trace.csv $O/prof/run_kernel_trace.csv 2>/dev/null | head -n 1)
python3 scripts/ktrace_steps.py "$f" 30 > $O/last_step_breakdown.txt 2>&1
head -n 34 $O/last_step_breakdown.txt
