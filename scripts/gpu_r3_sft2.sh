#!/bin/bash
# After the single-launch q+k RoPE and the complete-items flush trigger: GPU tests of the touched
# paths, then LLaMA-7B NB4 SFT (merged window) and its kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r3_sft2
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu \
  -k "rope or llama or merged or hf or sft or model or wgrad or overlapped" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
R=recipes/4_training_alpaca_deepspeed
COMMON="--data_path $O/alpaca.json --synthetic_examples 8192 --bf16 True --num_train_epochs 1 --model_max_length 512 \
 --learning_rate 2e-5 --warmup_ratio 0.03 --save_steps 100000 --tf32 False --report_to none --logging_steps 5 \
 --model_name_or_path llama-7b --deepspeed $R/configs/zero2_bf16.json --max_steps 40 \
 --per_device_train_batch_size 4 --gradient_accumulation_steps 8"
timeout -k 10 500 python -u $R/train.py $COMMON --output_dir /tmp/m1 > $O/llama_nb4.log 2>&1 || { tail -20 $O/llama_nb4.log; exit 1; }
echo "nb4: $(grep -o "'train_input_tokens_per_second'[^}]*" $O/llama_nb4.log | tail -1 | cut -c1-300)"
timeout -k 10 500 python -u $R/train.py $COMMON --output_dir /tmp/m2 --per_device_train_batch_size 32 --gradient_accumulation_steps 1 > $O/llama_mbs32.log 2>&1 || { tail -20 $O/llama_mbs32.log; exit 1; }
echo "mbs32: $(grep -o "'train_input_tokens_per_second'[^}]*" $O/llama_mbs32.log | tail -1 | cut -c1-300)"
