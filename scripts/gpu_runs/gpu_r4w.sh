#!/bin/bash
# Round 4: whole GPU suite + smoke after the row-split GEMMs / SP gather slots / async loopback
# stand-ins; LLaMA-7B NB4 SFT emulated DP8 rank with the loopback reduce-scatter / all-gather on a
# side stream (as RCCL's) vs in line; 1-GPU bench.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4w
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 3 "$R/$O/$name.log" | cut -c1-500
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step tests_gpu 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests
step smoke 180 python __graft_entry__.py smoke
SF=recipes/4_training_alpaca_deepspeed
COMMON="--data_path $O/alpaca.json --synthetic_examples 4096 --bf16 True --num_train_epochs 1 --model_max_length 512 \
 --learning_rate 2e-5 --warmup_ratio 0.03 --save_steps 100000 --tf32 False --report_to none --logging_steps 4 \
 --model_name_or_path llama-7b --deepspeed $SF/configs/zero2_bf16.json --per_device_train_batch_size 4 --gradient_accumulation_steps 8"
SMDT_EMULATE_DP=8 step llama_dp8_async 420 python -u $SF/train.py $COMMON --max_steps 24 --output_dir /tmp/m2
SMDT_LOOPBACK_ASYNC=0 SMDT_EMULATE_DP=8 step llama_dp8_inline 420 python -u $SF/train.py $COMMON --max_steps 24 --output_dir /tmp/m3
step bench 300 python bench.py --steps 20 --warmup 5
echo DONE
