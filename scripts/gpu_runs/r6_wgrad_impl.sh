# round 6: N = 1 bench with the weight gradients on the grouped MFMA kernel (default), on hipBLASLt
# (beta = 1, per weight), and per-shape timed (auto), alternated in one call
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r6_wgrad_impl; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
for i in 1 2; do
SMDT_WGRAD_IMPL=mfma run mfma_$i 300 python bench.py --steps 20 --warmup 5
SMDT_WGRAD_IMPL=blaslt run blaslt_$i 400 python bench.py --steps 20 --warmup 5
SMDT_WGRAD_IMPL=auto run auto_$i 400 python bench.py --steps 20 --warmup 5
done
echo DONE
