#!/bin/bash
# OPT-125m Alpaca SFT with the reference's DS config (ZeRO-3 + offload_param: cpu), NB4 batch
# (mbs 4 x GA 8): fused accumulation window (default) vs SMDT_SFT_FUSE_GA=0.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r3_opt_fused
mkdir -p $O
R=recipes/4_training_alpaca_deepspeed
export HSA_ENABLE_IPC_MODE_LEGACY=0
COMMON="--data_path $O/alpaca.json --synthetic_examples 8192 --bf16 True --num_train_epochs 1 --model_max_length 512 \
 --learning_rate 2e-5 --warmup_ratio 0.03 --save_steps 100000 --tf32 False --report_to none --logging_steps 5 \
 --per_device_train_batch_size 4 --gradient_accumulation_steps 8 --model_name_or_path facebook/opt-125m --max_steps 60 \
 --deepspeed $R/configs/default_offload_opt_param.json"
for v in 1 0; do
  SMDT_SFT_FUSE_GA=$v timeout -k 10 400 python -u $R/train.py $COMMON --output_dir /tmp/o$v > $O/opt125m_fuse$v.log 2>&1 \
    || { tail -20 $O/opt125m_fuse$v.log; exit 1; }
  echo "fuse=$v: $(grep -o "'train_runtime'[^}]*" $O/opt125m_fuse$v.log | tail -1 | cut -c1-400)"
done
