# round 6: relay tests (tune_sub with protocol resets, graph replay), GPT-3 tp4 stage with the
# ring gemm_tn routing gated on tile count, and the stand-in with a 16-workgroup transfer (what
# sub = 1 would give back)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/${OUT:-r6_relay_sub}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
run tests 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_relay.py
G="--emulate-tp 4 --hidden-size 4096 --num-attention-heads 32 --seq-length 2048 --micro-batch-size 4 --grad-accum 8 --tunableop 0 --steps 3 --warmup 2 --num-layers 16 --emulate-first-stage"
SMDT_LINK_STANDIN=192:32 run g0_standin_overlap 500 python bench.py $G
SMDT_LINK_STANDIN=192:32 SMDT_RING_GEMM_TN=0 run g0_standin_fill_only 500 python bench.py $G
ST="--emulate-tp 2 --micro-batch-size 32 --grad-accum 8 --steps 4 --warmup 2"
SMDT_LINK_STANDIN=256:16 run s0_16wg 400 python bench.py --num-layers 13 --emulate-first-stage $ST
SMDT_LINK_STANDIN=256:16 run s1_16wg 400 python bench.py --num-layers 11 --emulate-last-stage $ST
SMDT_LINK_STANDIN=256:32 run s0_32wg 400 python bench.py --num-layers 13 --emulate-first-stage $ST
echo DONE
