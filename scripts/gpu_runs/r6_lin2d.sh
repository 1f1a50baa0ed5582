# round 6: N = 1 bench A/B of the 2-D library call for 3-D linears (SMDT_LINEAR_2D), alternated
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r6_lin2d; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
for i in 1 2 3; do
SMDT_LINEAR_2D=1 run on_$i 300 python bench.py --steps 20 --warmup 5
SMDT_LINEAR_2D=0 run off_$i 300 python bench.py --steps 20 --warmup 5
done
echo DONE
