# round 6: where the queued W fillers pay most on the N = 8 stage rank under the relay stand-in
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r6_fillpass; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 SMDT_LINK_STANDIN=relay
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
N8="--emulate-tp 2 --micro-batch-size 32 --grad-accum 8 --num-layers 13 --emulate-first-stage --steps 6 --warmup 3"
run both_1 300 python bench.py $N8
SMDT_W_FILL_PASS=fwd run fwd 300 python bench.py $N8
SMDT_W_FILL_PASS=bwd run bwd 300 python bench.py $N8
SMDT_W_FILL_US_FWD=500 run both_fwd500 300 python bench.py $N8
SMDT_W_FILL_US_FWD=1000 run both_fwd1000 300 python bench.py $N8
SMDT_W_FILL_US=125 SMDT_W_FILL_US_FWD=500 run bwd125_fwd500 300 python bench.py $N8
run both_2 300 python bench.py $N8
echo DONE
