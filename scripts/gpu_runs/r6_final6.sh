# round 6, closing tree (Megatron flags, Switch MLP): N = 1 driver bench twice and smoke
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/${OUT:-r6_final6}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
run smoke 180 python __graft_entry__.py smoke
run bench 400 python bench.py --steps 20 --warmup 5
run bench_2 400 python bench.py --steps 20 --warmup 5
echo DONE
