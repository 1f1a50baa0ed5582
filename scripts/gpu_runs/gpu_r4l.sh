#!/bin/bash
# Round 4: full GPU tests + bench after the vision / loopback changes; the N = 8 stage emulation
# with 4 micro-batches of 64 (ring chunks at the N = 1 GEMM shapes); the LLaMA-7B SFT emulated
# DP8 rank again with the loopback reduce-scatter averaging like RCCL (no full-bucket scale);
# attention A/B of the dQ kernel's straight-line sub-tile pair (SMDT_FA_DQ_STRAIGHT).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4l
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 3 "$R/$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread
step bench 300 python bench.py --steps 20 --warmup 5
step attn 120 python benchmarks/bench_attention.py --b 64 --sdpa 0 --dropout 0.1
SMDT_FA_DQ_STRAIGHT=1 step attn_dq_straight 120 python benchmarks/bench_attention.py --b 64 --sdpa 0 --dropout 0.1
step attn2 120 python benchmarks/bench_attention.py --b 64 --sdpa 0 --dropout 0.1
SMDT_FA_DQ_STRAIGHT=1 step attn_dq_straight2 120 python benchmarks/bench_attention.py --b 64 --sdpa 0 --dropout 0.1
step predict_mb64 600 python -u benchmarks/predict_scaling.py --out $O/predict --only n1_dp tp2pp2_mb64_stage0 tp2pp2_mb64_stage1
SF=recipes/4_training_alpaca_deepspeed
COMMON="--data_path $O/alpaca.json --synthetic_examples 4096 --bf16 True --num_train_epochs 1 --model_max_length 512 \
 --learning_rate 2e-5 --warmup_ratio 0.03 --save_steps 100000 --tf32 False --report_to none --logging_steps 4 \
 --model_name_or_path llama-7b --deepspeed $SF/configs/zero2_bf16.json --per_device_train_batch_size 4 --gradient_accumulation_steps 8"
SMDT_EMULATE_DP=8 step llama_dp8_rank 420 python -u $SF/train.py $COMMON --max_steps 24 --output_dir /tmp/m2
step llama_n1 420 python -u $SF/train.py $COMMON --max_steps 24 --output_dir /tmp/m1
echo DONE
