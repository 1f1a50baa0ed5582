# Alpaca SFT on ONE GPU with the length-grouped attention: OPT-125m (NB4's DeepSpeed config, ZeRO-3
# + param offload) and LLaMA-7B ZeRO-2 (whole optimizer), each with the grouping on and off.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r5_sft_n1; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; grep -ho "'train_samples_per_second': [0-9.]*\|'train_input_tokens_per_second': [0-9.]*\|'train_mfu': [0-9.]*" $O/$n.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc; }
SF=$R/recipes/4_training_alpaca_deepspeed
C0="--data_path $O/alpaca.json --synthetic_examples 8192 --bf16 True --num_train_epochs 1 --model_max_length 512 \
 --learning_rate 2e-5 --warmup_ratio 0.03 --save_steps 100000 --tf32 False --report_to none --logging_steps 5"
OPT="$C0 --model_name_or_path facebook/opt-125m --deepspeed $SF/configs/default_offload_opt_param.json --per_device_train_batch_size 4 --gradient_accumulation_steps 8 --max_steps 40"
LL="$C0 --model_name_or_path llama-7b --deepspeed $SF/configs/zero2_bf16.json --per_device_train_batch_size 4 --gradient_accumulation_steps 8 --max_steps 16"
SMDT_SFT_LENGTH_GROUPS=0 run opt_off 600 python -u $SF/train.py $OPT --output_dir /tmp/o2
run opt_gated 600 python -u $SF/train.py $OPT --output_dir /tmp/o1
SMDT_SFT_LENGTH_GROUPS=force run opt_forced 600 python -u $SF/train.py $OPT --output_dir /tmp/o3
SMDT_SFT_LENGTH_GROUPS=0 run opt_off_2 600 python -u $SF/train.py $OPT --output_dir /tmp/o4
run opt_gated_2 600 python -u $SF/train.py $OPT --output_dir /tmp/o5
SMDT_SFT_LENGTH_GROUPS=force run opt_forced_2 600 python -u $SF/train.py $OPT --output_dir /tmp/o6
run llama_on 600 python -u $SF/train.py $LL --output_dir /tmp/l1
SMDT_SFT_LENGTH_GROUPS=0 run llama_off 600 python -u $SF/train.py $LL --output_dir /tmp/l2
echo DONE
