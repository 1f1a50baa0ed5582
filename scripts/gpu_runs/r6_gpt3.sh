# round 6: GPT-3 6.7B tp4 pp2 + SP stage rank (BASELINE config 5) under the paced link stand-in:
# the direct TP4 engine's 3-link rate (192 GB/s per ring step) with and without the exchange
# overlap (W fillers + grid-sized gemm_tn ring chunks)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/${OUT:-r6_gpt3}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
G="--emulate-tp 4 --hidden-size 4096 --num-attention-heads 32 --seq-length 2048 --micro-batch-size 4 --grad-accum 8 --tunableop 0 --steps 3 --warmup 2 --num-layers 16 --emulate-first-stage"
SMDT_W_FILL=0 SMDT_RING_GEMM_TN=0 run g0_copy 500 python bench.py $G
SMDT_LINK_STANDIN=192:32 SMDT_W_FILL=0 SMDT_RING_GEMM_TN=0 run g0_standin 500 python bench.py $G
SMDT_LINK_STANDIN=192:32 run g0_standin_overlap 500 python bench.py $G
echo DONE
