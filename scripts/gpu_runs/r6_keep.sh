# round 6: dropout keep words stored by the flash forward for the dQ kernel (SMDT_FA_KEEP_MASK):
# attention tests, then the N = 1 bench alternated on / off, then a kernel trace with it on
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r6_keep; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
run tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash or dropout"
for i in 1 2; do
SMDT_FA_KEEP_MASK=1 run on_$i 300 python bench.py --steps 20 --warmup 5
SMDT_FA_KEEP_MASK=0 run off_$i 300 python bench.py --steps 20 --warmup 5
done
cd /tmp
SMDT_FA_KEEP_MASK=1 run prof 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 3
cd $R
f=$(find $O/prof -name '*kernel_trace.csv' | head -n 1)
python scripts/ktrace_steps.py "$f" 40 > $O/last_step_breakdown.txt && head -n 12 $O/last_step_breakdown.txt
find $O/prof -name '*kernel_trace.csv' -delete
echo DONE
