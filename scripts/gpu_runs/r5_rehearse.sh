# One-GPU Gloo rehearsals of the multi-rank code paths of the round-5 tree (several ranks on ONE
# MI355X, RCCL refuses that): the pairs of the N = 8 layout (tp2pp2 + SP zbh2, tp2dp2 + SP,
# pp2dp2 zbh2) through bench.py, and the NB4 SFT path (ZeRO-2, 2 ranks, OPT-1.3B) with the
# length-grouped attention forced on. Step times are meaningless (Gloo stages CUDA tensors
# through the host); the point is that every path runs end to end with the real kernels.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r5_rehearse; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc; }
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --master-port 29533"
B="bench.py --steps 2 --warmup 1 --seqs-per-gpu 8 --micro-batch-size 4 --tunableop 0"
export SMDT_BENCH_BACKEND=gloo
run tp2pp2_zbh2 420 $TR --nproc-per-node 4 $B --gpus 4 --tp 2 --pp 2 --pp-schedule zbh2
run tp2dp2 420 $TR --nproc-per-node 4 $B --gpus 4 --tp 2 --pp 1
run pp2dp2_zbh2 420 $TR --nproc-per-node 4 $B --gpus 4 --tp 1 --pp 2 --pp-schedule zbh2
SF=$R/recipes/4_training_alpaca_deepspeed
SMDT_DIST_BACKEND=gloo SMDT_SFT_LENGTH_GROUPS=force run sft_opt13b_zero2 600 $TR --nproc-per-node 2 $SF/train.py \
 --data_path $O/alpaca.json --synthetic_examples 256 --bf16 True --num_train_epochs 1 --model_max_length 512 \
 --learning_rate 2e-5 --warmup_ratio 0.03 --save_steps 100000 --tf32 False --report_to none --logging_steps 1 \
 --model_name_or_path facebook/opt-1.3b --deepspeed $SF/configs/zero2_bf16.json --per_device_train_batch_size 4 \
 --gradient_accumulation_steps 2 --max_steps 3 --output_dir /tmp/r1
echo DONE
