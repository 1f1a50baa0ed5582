set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/${OUT:-r5_defer_add}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
run tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_graph_gpu.py -k "norm or layernorm or emulated or subbatch"
ST="--emulate-tp 2 --micro-batch-size 32 --grad-accum 8 --steps 6 --warmup 2"
for i in 1 2; do
  SMDT_DEFER_RS_ADD=0 run s1_off_$i 400 python bench.py --num-layers 11 --emulate-last-stage $ST
  run s1_on_$i 400 python bench.py --num-layers 11 --emulate-last-stage $ST
  SMDT_DEFER_RS_ADD=0 run s0_off_$i 400 python bench.py --num-layers 13 --emulate-first-stage $ST
  run s0_on_$i 400 python bench.py --num-layers 13 --emulate-first-stage $ST
done
run s1_on_graph 400 python bench.py --num-layers 11 --emulate-last-stage $ST --graph 1
if [ "${FULL:-0}" = "1" ]; then
  run pytest_gpu 900 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests
  run bench 400 python bench.py --steps 20 --warmup 5
fi
echo DONE
