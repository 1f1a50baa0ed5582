#!/bin/bash
# Round 4: LLaMA-7B NB4 SFT (ZeRO-2 bf16, mbs 4 x GA 8, fused window) on one MI355X, then ONE
# emulated rank of the 8-GPU ZeRO-2 job (SMDT_EMULATE_DP=8: its 1/8 optimizer shard and its share
# of the gradient reduce-scatter / parameter all-gather as local copies), then
# a rocprofv3 kernel trace of the emulated rank.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r4c
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=recipes/4_training_alpaca_deepspeed
COMMON="--data_path $O/alpaca.json --synthetic_examples 8192 --bf16 True --num_train_epochs 1 --model_max_length 512 \
 --learning_rate 2e-5 --warmup_ratio 0.03 --save_steps 100000 --tf32 False --report_to none --logging_steps 5 \
 --model_name_or_path llama-7b --deepspeed $R/configs/zero2_bf16.json --max_steps ${STEPS:-40} \
 --per_device_train_batch_size 4 --gradient_accumulation_steps 8"
timeout -k 10 500 python -u $R/train.py $COMMON --output_dir /tmp/m1 > $O/llama_n1.log 2>&1 || { tail -20 $O/llama_n1.log; exit 1; }
echo "n1: $(grep -o "'train_input_tokens_per_second'[^}]*" $O/llama_n1.log | tail -1 | cut -c1-300)"
SMDT_EMULATE_DP=8 timeout -k 10 500 python -u $R/train.py $COMMON --output_dir /tmp/m2 > $O/llama_dp8_rank.log 2>&1 || { tail -20 $O/llama_dp8_rank.log; exit 1; }
echo "dp8 rank: $(grep -o "'train_input_tokens_per_second'[^}]*" $O/llama_dp8_rank.log | tail -1 | cut -c1-400)"
cd /tmp
SMDT_EMULATE_DP=8 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/$R/train.py" $(echo $COMMON | sed "s#--data_path $O#--data_path $GRAFT_REPO_ROOT/$O#; s#$R/configs#$GRAFT_REPO_ROOT/$R/configs#; s#--max_steps [0-9]*#--max_steps 12#") \
  --output_dir /tmp/m3 > "$GRAFT_REPO_ROOT/$O/prof.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/$O/prof.log"; exit 1; }
echo DONE
