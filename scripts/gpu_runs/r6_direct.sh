# round 6: GPT-3 6.7B tp4 pp2 + SP stage rank (BASELINE config 5) with the TP4 exchanges through
# a paced stand-in of the direct multi-link engine (row pieces over 3 links at 64 GB/s each,
# SMDT_LINK_STANDIN=direct) against the ring stand-in at the same aggregate rate (192 GB/s a step)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/${OUT:-r6_direct}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
run test 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_parallel_gpu.py -k "direct_engine_standin or w_fillers"
G="--emulate-tp 4 --hidden-size 4096 --num-attention-heads 32 --seq-length 2048 --micro-batch-size 4 --grad-accum 8 --tunableop 0 --steps 3 --warmup 2 --num-layers 16 --emulate-first-stage"
if [ "${PASS:-1}" = 1 ]; then
SMDT_LINK_STANDIN=192:32 run g0_ring_overlap 500 python bench.py $G
SMDT_LINK_STANDIN=direct:64:32 run g0_direct_overlap 500 python bench.py $G
SMDT_LINK_STANDIN=direct:64:32 SMDT_W_FILL=0 SMDT_RING_GEMM_TN=0 run g0_direct_nofill 500 python bench.py $G
SMDT_LINK_STANDIN=direct:64:32 SMDT_TP_DIRECT_PIECES=4 run g0_direct_p4 500 python bench.py $G
elif [ "${PASS:-1}" = 5 ]; then
# pass 5: row pieces with the per-peer GEMMs concurrent on side streams (SMDT_TP_DIRECT_CONCURRENT)
run test5 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_parallel_gpu.py -k "direct_engine_standin"
SMDT_LINK_STANDIN=direct:64:32 SMDT_TP_DIRECT_PIECES=1 run g0_p1_d 500 python bench.py $G
SMDT_LINK_STANDIN=direct:64:32 SMDT_TP_DIRECT_PIECES=2 run g0_p2_conc 500 python bench.py $G
SMDT_LINK_STANDIN=direct:64:32 SMDT_TP_DIRECT_PIECES=4 run g0_p4_conc 500 python bench.py $G
SMDT_LINK_STANDIN=direct:64:32 SMDT_TP_DIRECT_PIECES=2 SMDT_TP_DIRECT_CONCURRENT=0 run g0_p2_seq 500 python bench.py $G
SMDT_TP_DIRECT_PIECES=2 run g0_p2_conc_nolink 500 python bench.py $G
elif [ "${PASS:-1}" = 6 ]; then
# pass 6: the same with 16 hardware queues per process (HIP's default is 4: streams beyond share
# queues, so a side stream can queue behind a paced copy that spins for its link time)
N8="--emulate-tp 2 --micro-batch-size 32 --grad-accum 8 --num-layers 13 --emulate-first-stage --steps 6 --warmup 3"
GPU_MAX_HW_QUEUES=16 SMDT_LINK_STANDIN=direct:64:32 SMDT_TP_DIRECT_PIECES=2 run q16_g0_p2_conc 500 python bench.py $G
GPU_MAX_HW_QUEUES=16 SMDT_LINK_STANDIN=direct:64:32 SMDT_TP_DIRECT_PIECES=1 run q16_g0_p1 500 python bench.py $G
GPU_MAX_HW_QUEUES=16 SMDT_LINK_STANDIN=relay run q16_s0_relay 300 python bench.py $N8
SMDT_LINK_STANDIN=relay run q4_s0_relay 300 python bench.py $N8
GPU_MAX_HW_QUEUES=16 run q16_n1 300 python bench.py --steps 20 --warmup 5
run q4_n1 300 python bench.py --steps 20 --warmup 5
elif [ "${PASS:-1}" = 4 ]; then
# pass 4: the interleave's short phases on a chain stream per half (SMDT_SP_SUBBATCH_CHAIN=1)
run test4 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_parallel_gpu.py tests/test_graph_gpu.py -k "direct_engine_standin or subbatch"
SMDT_LINK_STANDIN=direct:64:32 SMDT_TP_DIRECT_PIECES=1 SMDT_SP_SUBBATCH=2 run g0_direct_p1_chain 500 python bench.py $G
SMDT_LINK_STANDIN=direct:64:32 SMDT_TP_DIRECT_PIECES=1 run g0_direct_p1_c 500 python bench.py $G
N8="--emulate-tp 2 --micro-batch-size 32 --grad-accum 8 --num-layers 13 --emulate-first-stage --steps 6 --warmup 3"
SMDT_LINK_STANDIN=relay run s0_relay 300 python bench.py $N8
SMDT_LINK_STANDIN=relay SMDT_SP_SUBBATCH=2 run s0_relay_chain 300 python bench.py $N8
SMDT_LINK_STANDIN=relay SMDT_SP_SUBBATCH=2 SMDT_SP_SUBBATCH_CHAIN=0 run s0_relay_sub_inline 300 python bench.py $N8
elif [ "${PASS:-1}" = 3 ]; then
# pass 3: whole chunks (merged peer GEMMs) with and without the sub-batch interleave over the engine
SMDT_LINK_STANDIN=direct:64:32 SMDT_TP_DIRECT_PIECES=1 run g0_direct_p1_b 500 python bench.py $G
SMDT_LINK_STANDIN=direct:64:32 SMDT_TP_DIRECT_PIECES=1 SMDT_SP_SUBBATCH=2 run g0_direct_p1_sub2 500 python bench.py $G
SMDT_LINK_STANDIN=direct:64:32 SMDT_TP_DIRECT_PIECES=2 SMDT_SP_SUBBATCH=2 run g0_direct_p2_sub2 500 python bench.py $G
SMDT_LINK_STANDIN=direct:64:32 SMDT_TP_DIRECT_PIECES=1 SMDT_SP_SUBBATCH=2 run g1_direct_p1_sub2 500 python bench.py ${G/--emulate-first-stage/--emulate-last-stage}
SMDT_LINK_STANDIN=direct:64:32 SMDT_TP_DIRECT_PIECES=1 run g1_direct_p1 500 python bench.py ${G/--emulate-first-stage/--emulate-last-stage}
else
# pass 2: the ring at ONE link's rate (what a real TP4 ring gets: one link per direction per step)
SMDT_LINK_STANDIN=64:32 run g0_ring1link_overlap 500 python bench.py $G
SMDT_LINK_STANDIN=direct:64:32 SMDT_TP_DIRECT_PIECES=1 run g0_direct_p1 500 python bench.py $G
SMDT_LINK_STANDIN=direct:64:32 run g0_direct_p2_again 500 python bench.py $G
SMDT_LINK_STANDIN=192:32 run g0_ring_overlap_again 500 python bench.py $G
fi
echo DONE
