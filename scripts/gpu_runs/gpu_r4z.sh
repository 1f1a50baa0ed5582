#!/bin/bash
# Round 4: GPU suite after the wgrad overwrite mode / lazily zeroed ZeRO-2 buffers / fused-norm
# gather waits; LLaMA-7B NB4 SFT emulated DP8 rank A/B (SMDT_LAZY_GRAD_ZERO); 1-GPU bench; the
# per-call durations of the bench step's GEMMs.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4z
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
SF=recipes/4_training_alpaca_deepspeed
COMMON="--data_path $O/alpaca.json --synthetic_examples 4096 --bf16 True --num_train_epochs 1 --model_max_length 512 \
 --learning_rate 2e-5 --warmup_ratio 0.03 --save_steps 100000 --tf32 False --report_to none --logging_steps 4 \
 --model_name_or_path llama-7b --deepspeed $SF/configs/zero2_bf16.json --per_device_train_batch_size 4 --gradient_accumulation_steps 8"
SMDT_EMULATE_DP=8 step llama_dp8_lazy 420 python -u $SF/train.py $COMMON --max_steps 24 --output_dir /tmp/m2
SMDT_LAZY_GRAD_ZERO=0 SMDT_EMULATE_DP=8 step llama_dp8_zeroed 420 python -u $SF/train.py $COMMON --max_steps 24 --output_dir /tmp/m3
SMDT_EMULATE_DP=8 step llama_dp8_lazy2 420 python -u $SF/train.py $COMMON --max_steps 24 --output_dir /tmp/m4
step bench 300 python bench.py --steps 20 --warmup 5
bash scripts/gpu_runs/gpu_r4y.sh > "$O/r4y.out" 2>&1 || echo "r4y rc=$?"
cp -r gpurun_out/r4y "$O/" 2>/dev/null
echo DONE
