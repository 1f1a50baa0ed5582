#!/bin/bash
# Merged gradient-accumulation window for the deferred wgrad: equivalence test, then LLaMA-7B
# Alpaca SFT at the NB4 config (mbs 4 x GA 8, ZeRO-2, padding-free) with the window on / off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r3_merge
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_parallel_gpu.py \
  -k "merged_accumulation or overlapped or wgrad" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
R=recipes/4_training_alpaca_deepspeed
COMMON="--data_path $O/alpaca.json --synthetic_examples 8192 --bf16 True --num_train_epochs 1 --model_max_length 512 \
 --learning_rate 2e-5 --warmup_ratio 0.03 --save_steps 100000 --tf32 False --report_to none --logging_steps 5 \
 --model_name_or_path llama-7b --deepspeed $R/configs/zero2_bf16.json --max_steps 40 \
 --per_device_train_batch_size 4 --gradient_accumulation_steps 8"
for v in 1 0; do
  SMDT_WGRAD_MERGE_ACCUM=$v timeout -k 10 500 python -u $R/train.py $COMMON --output_dir /tmp/m$v > $O/llama_nb4_merge$v.log 2>&1 \
    || { tail -20 $O/llama_nb4_merge$v.log; exit 1; }
  echo "merge=$v: $(grep -o "'train_input_tokens_per_second'[^}]*" $O/llama_nb4_merge$v.log | tail -1 | cut -c1-300)"
done
