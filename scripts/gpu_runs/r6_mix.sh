# round 6: fused-MLP chip-fill gate check (GPT-3 tp4 stage), filler implementation A/B under the
# paced stand-in, the affected GPU tests, then the secondary-recipe refresh (r6_recipes.sh)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/${OUT:-r6_mix}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
run tests 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gemm_tn_gpu.py tests/test_parallel_gpu.py
G="--emulate-tp 4 --hidden-size 4096 --num-attention-heads 32 --seq-length 2048 --micro-batch-size 4 --grad-accum 8 --tunableop 0 --steps 3 --warmup 2 --num-layers 16 --emulate-first-stage"
SMDT_W_FILL=0 SMDT_RING_GEMM_TN=0 run g0_copy 500 python bench.py $G
SMDT_LINK_STANDIN=192:32 run g0_standin_overlap 500 python bench.py $G
SMDT_LINK_STANDIN=192:32 SMDT_W_FILL=0 SMDT_RING_GEMM_TN=0 run g0_standin 500 python bench.py $G
ST="--emulate-tp 2 --micro-batch-size 32 --grad-accum 8 --steps 4 --warmup 2"
SMDT_LINK_STANDIN=relay run s0_fill_grouped 400 python bench.py --num-layers 13 --emulate-first-stage $ST
SMDT_LINK_STANDIN=relay SMDT_W_FILL_IMPL=blaslt run s0_fill_blaslt 400 python bench.py --num-layers 13 --emulate-first-stage $ST
SMDT_LINK_STANDIN=relay run s1_fill_grouped 400 python bench.py --num-layers 11 --emulate-last-stage $ST
SMDT_LINK_STANDIN=relay SMDT_W_FILL_IMPL=blaslt run s1_fill_blaslt 400 python bench.py --num-layers 11 --emulate-last-stage $ST
echo DONE
