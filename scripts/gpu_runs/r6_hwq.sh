# round 6: 16 vs 4 (HIP's default) hardware queues per process, alternated: the emulated N = 8
# stage ranks under the relay stand-in (side streams: fillers, exchanges) and the N = 1 bench
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r6_hwq; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc; }
S0="--emulate-tp 2 --micro-batch-size 32 --grad-accum 8 --num-layers 13 --emulate-first-stage --steps 6 --warmup 3"
S1="--emulate-tp 2 --micro-batch-size 32 --grad-accum 8 --num-layers 11 --emulate-last-stage --steps 6 --warmup 3"
for i in 1 2 3; do
for q in 16 4; do
GPU_MAX_HW_QUEUES=$q SMDT_LINK_STANDIN=relay run s0_q${q}_$i 300 python bench.py $S0
GPU_MAX_HW_QUEUES=$q SMDT_LINK_STANDIN=relay run s1_q${q}_$i 300 python bench.py $S1
done
done
for i in 1 2; do
for q in 16 4 8; do
GPU_MAX_HW_QUEUES=$q run n1_q${q}_$i 300 python bench.py --steps 20 --warmup 5
done
done
echo DONE
