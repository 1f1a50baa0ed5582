# Emulated N = 8 last-stage rank: the loopback ring exchange in line on the compute stream (default)
# vs on the loopback group's high-priority side stream (SMDT_LOOPBACK_RING_ASYNC=1), interleaved,
# eager; then the async arm under a whole-step HIP graph.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r5_lb_async; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
ST="--num-layers 11 --emulate-last-stage --emulate-tp 2 --micro-batch-size 32 --grad-accum 8 --steps 6 --warmup 2"
for i in 1 2; do
  run inline_$i 400 python bench.py $ST
  SMDT_LOOPBACK_RING_ASYNC=1 run async_$i 400 python bench.py $ST
done
run inline_graph 400 python bench.py $ST --graph 1
SMDT_LOOPBACK_RING_ASYNC=1 run async_graph 400 python bench.py $ST --graph 1
echo DONE
