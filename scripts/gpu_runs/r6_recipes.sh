# round 6: refresh of the secondary recipes on the round-6 tree:
# Oxford-Pet ResNet-50 / swin_b as one emulated dp8 rank (graphed and eager), Alpaca OPT-125m with
# the reference's own ZeRO-3 + offload DeepSpeed JSON (+ a kernel trace of it), LLaMA-7B ZeRO-2 as
# one emulated rank of the 8-GPU job
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/${OUT:-r6_recipes}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 2 $O/$n.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
V="--model resnet50 --size 224 --batch 64 --steps 20 --warmup 5 --emulate-dp 8"
run r50_dp8_graph 500 python benchmarks/bench_vision.py $V --graph 1
run r50_dp8_eager 500 python benchmarks/bench_vision.py $V --graph 0
S="--model swin_b --size 128 --batch 40 --steps 20 --warmup 5 --emulate-dp 8"
run swin_dp8_graph 500 python benchmarks/bench_vision.py $S --graph 1
SF=$R/recipes/4_training_alpaca_deepspeed
C0="--data_path $O/alpaca.json --synthetic_examples 4096 --bf16 True --num_train_epochs 1 \
 --learning_rate 2e-5 --warmup_ratio 0.03 --save_steps 100000 --tf32 False --report_to none --logging_steps 4"
run opt125m_zero3_offload 500 python -u $SF/train.py $C0 --model_name_or_path facebook/opt-125m --output_dir /tmp/o1 \
  --per_device_train_batch_size 4 --gradient_accumulation_steps 8 --max_steps 40 --deepspeed $SF/configs/default_offload_opt_param.json
cd /tmp
run opt125m_prof 500 rocprofv3 --kernel-trace --stats -d $O/opt_prof -o run --output-format csv -- python3 -u $SF/train.py $C0 \
  --model_name_or_path facebook/opt-125m --output_dir /tmp/o2 --per_device_train_batch_size 4 --gradient_accumulation_steps 8 \
  --max_steps 12 --deepspeed $SF/configs/default_offload_opt_param.json
cd $R
f=$(find $O/opt_prof -name '*kernel_trace.csv' | head -n 1)
python scripts/ktrace_steps.py "$f" 30 > $O/opt_last_step_breakdown.txt 2>&1; head -n 12 $O/opt_last_step_breakdown.txt
find $O/opt_prof -name '*kernel_trace.csv' -delete
C1="$C0 --model_max_length 512 --model_name_or_path llama-7b --deepspeed $SF/configs/zero2_bf16.json \
 --per_device_train_batch_size 4 --gradient_accumulation_steps 8"
SMDT_EMULATE_DP=8 run llama_dp8 500 python -u $SF/train.py $C1 --max_steps 24 --output_dir /tmp/m1
echo DONE
