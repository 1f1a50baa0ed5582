set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r5_prio; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 2 $O/$n.log | cut -c1-700; [ $rc -eq 0 ] || exit $rc; }
run pytest_kernels 600 python -u -m pytest -q -x --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_model_gpu.py
run prio 300 python benchmarks/bench_comm_priority.py
run stage1_high 400 python bench.py --steps 6 --warmup 2 --num-layers 11 --emulate-last-stage --emulate-tp 2 --micro-batch-size 32 --grad-accum 8
SMDT_COMM_PRIORITY=normal run stage1_normal 400 python bench.py --steps 6 --warmup 2 --num-layers 11 --emulate-last-stage --emulate-tp 2 --micro-batch-size 32 --grad-accum 8
run stage1_high2 400 python bench.py --steps 6 --warmup 2 --num-layers 11 --emulate-last-stage --emulate-tp 2 --micro-batch-size 32 --grad-accum 8
echo DONE
