#!/bin/bash
# Overlapped optimizer step: equivalence test, GPT bench, LLaMA SFT (on / off).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r3_optov
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_parallel_gpu.py tests/test_kernels_gpu.py -x -q -k "overlapped or dgrad_weight_t" \
  --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 1 0; do
  SMDT_OVERLAP_OPTIMIZER=$v timeout -k 10 300 python bench.py --steps 10 --warmup 4 > $O/bench_ov$v.log 2>&1 || { tail -20 $O/bench_ov$v.log; exit 1; }
  echo "bench ov=$v $(grep '^{' $O/bench_ov$v.log | tail -1 | cut -c1-160)"
done
R=recipes/4_training_alpaca_deepspeed
COMMON="--data_path $O/alpaca.json --synthetic_examples 8192 --bf16 True --num_train_epochs 1 --model_max_length 512 \
 --learning_rate 2e-5 --warmup_ratio 0.03 --save_steps 100000 --tf32 False --report_to none --logging_steps 5 \
 --model_name_or_path llama-7b --deepspeed $R/configs/zero2_bf16.json --max_steps 60 \
 --per_device_train_batch_size 32 --gradient_accumulation_steps 1"
for v in 1 0; do
  SMDT_OVERLAP_OPTIMIZER=$v timeout -k 10 600 python -u $R/train.py $COMMON --output_dir /tmp/c$v > $O/llama_ov$v.log 2>&1 \
    || { tail -20 $O/llama_ov$v.log; exit 1; }
  echo "llama mbs32 ov=$v: $(grep -o "'train_input_tokens_per_second'[^}]*" $O/llama_ov$v.log | tail -1)"
done
