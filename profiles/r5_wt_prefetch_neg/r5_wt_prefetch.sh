# dgrad W^T made ahead on a side stream (SMDT_DGRAD_WT_PREFETCH): tests, N = 1 bench A/B, SFT rank A/B.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r5_wt_prefetch; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
run tests 900 python -u -m pytest -q -x --timeout 150 --timeout-method thread -m gpu tests/test_model_gpu.py tests/test_graph_gpu.py tests/test_parallel_gpu.py tests/test_sft.py tests/test_hf_models.py
for i in 1 2; do
  run bench_on_$i 300 python bench.py --steps 15 --warmup 3
  SMDT_DGRAD_WT_PREFETCH=0 run bench_off_$i 300 python bench.py --steps 15 --warmup 3
done
SF=$R/recipes/4_training_alpaca_deepspeed
COMMON="--data_path $O/alpaca.json --synthetic_examples 4096 --bf16 True --num_train_epochs 1 --model_max_length 512 \
 --learning_rate 2e-5 --warmup_ratio 0.03 --save_steps 100000 --tf32 False --report_to none --logging_steps 4 \
 --model_name_or_path llama-7b --deepspeed $SF/configs/zero2_bf16.json --per_device_train_batch_size 4 --gradient_accumulation_steps 8"
for i in 1 2; do
  SMDT_EMULATE_DP=8 run sft_on_$i 420 python -u $SF/train.py $COMMON --max_steps 24 --output_dir /tmp/m$i
  SMDT_DGRAD_WT_PREFETCH=0 SMDT_EMULATE_DP=8 run sft_off_$i 420 python -u $SF/train.py $COMMON --max_steps 24 --output_dir /tmp/n$i
done
grep -ho "'train_input_tokens_per_second': [0-9.]*\|'train_mfu': [0-9.]*" $O/sft_*.log
echo DONE
