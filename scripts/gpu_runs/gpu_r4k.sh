#!/bin/bash
# Round 4: vision with whole-step HIP-graph capture (A/B against eager, ResNet-50 224 and swin_b
# 128), then the LLaMA-7B NB4 SFT: 1 GPU and one emulated rank of the 8-GPU ZeRO-2 job
# (SMDT_EMULATE_DP=8: its 1/8 optimizer shard + loopback reduce-scatter / all-gather), with a
# kernel trace of the emulated rank.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4k
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
step r50_eager 400 python benchmarks/bench_vision.py --model resnet50 --size 224 --batch 64 --steps 20 --warmup 5
step r50_graph 300 python benchmarks/bench_vision.py --model resnet50 --size 224 --batch 64 --steps 20 --warmup 5 --graph 1 --miopen-prewarm 0
step swin_eager 300 python benchmarks/bench_vision.py --model swin_b --size 128 --batch 40 --steps 20 --warmup 5
step swin_graph 300 python benchmarks/bench_vision.py --model swin_b --size 128 --batch 40 --steps 20 --warmup 5 --graph 1 --miopen-prewarm 0
SF=recipes/4_training_alpaca_deepspeed
COMMON="--data_path $O/alpaca.json --synthetic_examples 4096 --bf16 True --num_train_epochs 1 --model_max_length 512 \
 --learning_rate 2e-5 --warmup_ratio 0.03 --save_steps 100000 --tf32 False --report_to none --logging_steps 4 \
 --model_name_or_path llama-7b --deepspeed $SF/configs/zero2_bf16.json --per_device_train_batch_size 4 --gradient_accumulation_steps 8"
step llama_n1 420 python -u $SF/train.py $COMMON --max_steps 16 --output_dir /tmp/m1
SMDT_EMULATE_DP=8 step llama_dp8_rank 420 python -u $SF/train.py $COMMON --max_steps 16 --output_dir /tmp/m2
cd /tmp
SMDT_EMULATE_DP=8 step llama_dp8_prof 420 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_llama_dp8" -o run --output-format csv -- \
  python3 "$R/$SF/train.py" $(echo $COMMON | sed "s#--data_path $O#--data_path $R/$O#; s#$SF/configs#$R/$SF/configs#") \
  --max_steps 6 --output_dir /tmp/m3
echo DONE
