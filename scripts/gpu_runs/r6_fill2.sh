# round 6: W fillers v2 (time budget per wait, backward waits too) under the paced relay stand-in
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/${OUT:-r6_fill2}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 SMDT_LINK_STANDIN=relay SMDT_W_FILL=1
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
ST="--emulate-tp 2 --micro-batch-size 32 --grad-accum 8 --steps 4 --warmup 2"
for S in s0 s1; do
  if [ $S = s0 ]; then SA="--num-layers 13 --emulate-first-stage"; else SA="--num-layers 11 --emulate-last-stage"; fi
  run ${S}_fill_blaslt 400 python bench.py $SA $ST
  SMDT_RING_GEMM_TN=1 run ${S}_fill_tn 400 python bench.py $SA $ST
  SMDT_W_FILL_US=60 run ${S}_fill60 400 python bench.py $SA $ST
  SMDT_W_FILL_US=200 run ${S}_fill200 400 python bench.py $SA $ST
done
echo DONE
