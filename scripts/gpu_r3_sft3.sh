#!/bin/bash
# Fused GA window in the SFT trainer: LLaMA-7B NB4 SFT fused (default) vs SMDT_SFT_FUSE_GA=0.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r3_sft3
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu -k "merged or sft or hf" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
R=recipes/4_training_alpaca_deepspeed
COMMON="--data_path $O/alpaca.json --synthetic_examples 8192 --bf16 True --num_train_epochs 1 --model_max_length 512 \
 --learning_rate 2e-5 --warmup_ratio 0.03 --save_steps 100000 --tf32 False --report_to none --logging_steps 5 \
 --model_name_or_path llama-7b --deepspeed $R/configs/zero2_bf16.json --max_steps 40 \
 --per_device_train_batch_size 4 --gradient_accumulation_steps 8"
timeout -k 10 500 python -u $R/train.py $COMMON --output_dir /tmp/m1 > $O/llama_nb4.log 2>&1 || { tail -20 $O/llama_nb4.log; exit 1; }
echo "nb4: $(grep -o "'train_input_tokens_per_second'[^}]*" $O/llama_nb4.log | tail -1 | cut -c1-300)"
SMDT_SFT_FUSE_GA=0 timeout -k 10 500 python -u $R/train.py $COMMON --output_dir /tmp/m2 > $O/llama_nb4_unfused.log 2>&1 || { tail -20 $O/llama_nb4_unfused.log; exit 1; }
echo "nb4 unfused: $(grep -o "'train_input_tokens_per_second'[^}]*" $O/llama_nb4_unfused.log | tail -1 | cut -c1-300)"
