# round 6: GPU checks of the deferred-summand ledger, the fused-MLP gather wait and the emulated
# stage ranks (eager) on the changed tree
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/${OUT:-r6_check}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
run tests 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu ${TESTS:-tests/test_parallel_gpu.py tests/test_graph_gpu.py tests/test_model_gpu.py}
ST="--emulate-tp 2 --micro-batch-size 32 --grad-accum 8 --steps 4 --warmup 2"
run s0 400 python bench.py --num-layers 13 --emulate-first-stage $ST
run s1 400 python bench.py --num-layers 11 --emulate-last-stage $ST
echo DONE
