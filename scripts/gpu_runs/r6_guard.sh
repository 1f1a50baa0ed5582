# round 6: the forward guard on deferred reduce-scatter summands (PendingPartial): full GPU suite
# and the N = 8 stage rank under the relay stand-in, guard on / off
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r6_guard; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
if [ "${TESTS:-1}" = 1 ]; then run pytest_gpu 900 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests; fi
S0="--emulate-tp 2 --micro-batch-size 32 --grad-accum 8 --num-layers 13 --emulate-first-stage --steps 6 --warmup 3"
for i in 1 2 3; do
SMDT_LINK_STANDIN=relay run s0_guard_$i 300 python bench.py $S0
SMDT_LINK_STANDIN=relay SMDT_DEFER_RS_GUARD=0 run s0_noguard_$i 300 python bench.py $S0
done
run n1 300 python bench.py --steps 20 --warmup 5
echo DONE
