#!/bin/bash
# Round 4: token-per-block RoPE kernel — GPU tests, SFT emulated DP8 rank (LLaMA-7B, RoPE on
# 64 heads of 128) before / after in one call (SMDT_ROPE_GRIDSTRIDE=1 forces the old kernel).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4aj
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 2 "$R/$O/$name.log" | cut -c1-500
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_hf_models.py
SF=recipes/4_training_alpaca_deepspeed
COMMON="--data_path $O/alpaca.json --synthetic_examples 4096 --bf16 True --num_train_epochs 1 --model_max_length 512 \
 --learning_rate 2e-5 --warmup_ratio 0.03 --save_steps 100000 --tf32 False --report_to none --logging_steps 4 \
 --model_name_or_path llama-7b --deepspeed $SF/configs/zero2_bf16.json --per_device_train_batch_size 4 --gradient_accumulation_steps 8"
SMDT_EMULATE_DP=8 step llama_dp8_tok 420 python -u $SF/train.py $COMMON --max_steps 24 --output_dir /tmp/m2
SMDT_ROPE_GRIDSTRIDE=1 SMDT_EMULATE_DP=8 step llama_dp8_grid 420 python -u $SF/train.py $COMMON --max_steps 24 --output_dir /tmp/m3
SMDT_EMULATE_DP=8 step llama_dp8_tok2 420 python -u $SF/train.py $COMMON --max_steps 24 --output_dir /tmp/m4
echo DONE
