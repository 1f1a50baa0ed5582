# round 6, closing tree: full GPU suite, smoke, N = 1 bench, and pretrain_gpt on the GPU with
# --optimizer sgd and with the Megatron params-norm / num-zeros log fields
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/${OUT:-r6_final5}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
export WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1
G="recipes/3_training_megatron-lm/pretrain_gpt.py --num-layers 4 --hidden-size 512 --num-attention-heads 8 \
 --seq-length 512 --max-position-embeddings 512 --micro-batch-size 4 --global-batch-size 8 --lr 0.01 \
 --lr-warmup-iters 1 --mock-data --log-interval 1 --eval-interval 100 --eval-iters 1 --vocab-size 8192 \
 --tokenizer-type NullTokenizer --train-iters 6 --bf16 --log-params-norm --log-num-zeros-in-grad"
MASTER_PORT=29551 run pretrain_adam 300 python $G
MASTER_PORT=29552 run pretrain_sgd 300 python $G --optimizer sgd --sgd-momentum 0.9
unset WORLD_SIZE RANK LOCAL_RANK MASTER_ADDR
run pytest_gpu 900 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests
run smoke 180 python __graft_entry__.py smoke
run bench 400 python bench.py --steps 20 --warmup 5
echo DONE
