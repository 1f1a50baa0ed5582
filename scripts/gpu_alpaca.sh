#!/bin/bash
# Alpaca SFT on one MI355X: OPT-125m (reference NB4 config, bf16) then LLaMA-7B ZeRO-2 bf16.
set -o pipefail
mkdir -p gpurun_out/alpaca
R=recipes/4_training_alpaca_deepspeed
COMMON="--data_path gpurun_out/alpaca/alpaca.json --synthetic_examples ${NEX:-8192} --bf16 True --num_train_epochs 1 \
 --learning_rate 2e-5 --warmup_ratio 0.03 --save_steps 100000 --tf32 False --report_to none --logging_steps 5"
timeout -k 10 ${T1:-600} python $R/train.py --model_name_or_path facebook/opt-125m --output_dir /tmp/alp_opt \
  --per_device_train_batch_size ${MBS:-4} --gradient_accumulation_steps ${GA:-8} --max_steps ${STEPS:-40} \
  --deepspeed $R/configs/default_offload_opt_param.json $COMMON $EXTRA > gpurun_out/alpaca/opt125m.log 2>&1
rc=$?; tail -3 gpurun_out/alpaca/opt125m.log; echo "opt rc=$rc"
[ $rc -ne 0 ] && exit $rc
if [ -n "$LLAMA" ]; then
  timeout -k 10 ${T2:-600} python $R/train.py --model_name_or_path llama-7b --output_dir /tmp/alp_llama \
    --per_device_train_batch_size ${LMBS:-4} --gradient_accumulation_steps 1 --max_steps ${LSTEPS:-8} \
    --deepspeed $R/configs/zero2_bf16.json $COMMON > gpurun_out/alpaca/llama7b.log 2>&1
  rc=$?; tail -3 gpurun_out/alpaca/llama7b.log; echo "llama rc=$rc"
fi
exit $rc
