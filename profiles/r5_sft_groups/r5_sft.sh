# LLaMA-7B NB4 SFT (ZeRO-2 bf16, 4 x GA 8): one emulated rank of the 8-GPU job, twice, then a
# kernel trace of a short run and its last-step breakdown.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r5_sft; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 2 $O/$n.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
SF=$R/recipes/4_training_alpaca_deepspeed
COMMON="--data_path $O/alpaca.json --synthetic_examples 4096 --bf16 True --num_train_epochs 1 --model_max_length 512 \
 --learning_rate 2e-5 --warmup_ratio 0.03 --save_steps 100000 --tf32 False --report_to none --logging_steps 4 \
 --model_name_or_path llama-7b --deepspeed $SF/configs/zero2_bf16.json --per_device_train_batch_size 4 --gradient_accumulation_steps 8"
run tests 600 python -u -m pytest -q -x --timeout 150 --timeout-method thread -m gpu tests/test_hf_models.py tests/test_sft.py
SMDT_EMULATE_DP=8 run llama_dp8 420 python -u $SF/train.py $COMMON --max_steps 24 --output_dir /tmp/m1
SMDT_SFT_LENGTH_GROUPS=0 SMDT_EMULATE_DP=8 run llama_dp8_nogroups 420 python -u $SF/train.py $COMMON --max_steps 24 --output_dir /tmp/m2
SMDT_EMULATE_DP=8 run llama_dp8_2 420 python -u $SF/train.py $COMMON --max_steps 24 --output_dir /tmp/m4
SMDT_SFT_LENGTH_GROUPS=0 SMDT_EMULATE_DP=8 run llama_dp8_nogroups_2 420 python -u $SF/train.py $COMMON --max_steps 24 --output_dir /tmp/m5
cd /tmp
SMDT_EMULATE_DP=8 run prof 420 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u $SF/train.py $COMMON --max_steps 8 --output_dir /tmp/m3
cd $R
f=$(find $O/prof -name '*kernel_trace.csv' | head -n 1)
python scripts/ktrace_steps.py "$f" 45 > $O/last_step_breakdown.txt 2>&1 && head -n 30 $O/last_step_breakdown.txt
find $O/prof -name '*kernel_trace.csv' -delete
echo DONE
