#!/bin/bash
# Round-2 GPU session B: model-level GPU tests, then the reference Alpaca config (OPT-125m, ZeRO-3 +
# offload_param + offload_optimizer) on the true stage-3 path, then ZeRO-3 without offload.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/alpaca
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 12 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
R=recipes/4_training_alpaca_deepspeed
COMMON="--data_path gpurun_out/alpaca/alpaca.json --synthetic_examples 4096 --bf16 True --num_train_epochs 1 \
 --learning_rate 2e-5 --warmup_ratio 0.03 --save_steps 100000 --tf32 False --report_to none --logging_steps 5"
step pytest_model 300 python -u -m pytest tests/test_model_gpu.py tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread
step opt125m_zero3_offload 400 python $R/train.py --model_name_or_path facebook/opt-125m --output_dir /tmp/alp_opt \
  --per_device_train_batch_size 4 --gradient_accumulation_steps 8 --max_steps 20 \
  --deepspeed $R/configs/default_offload_opt_param.json $COMMON
step opt125m_zero3_hbm 400 python $R/train.py --model_name_or_path facebook/opt-125m --output_dir /tmp/alp_opt2 \
  --per_device_train_batch_size 4 --gradient_accumulation_steps 8 --max_steps 20 \
  --deepspeed $R/configs/zero3_bf16.json $COMMON
echo DONE
