# round 6: W fillers in the forward exchange waits (SMDT_W_FILL=1) on the emulated stage ranks
# under the paced relay stand-in, with the CU reservation (default) and ring chunks on gemm_tn
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/${OUT:-r6_fill}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
ST="--emulate-tp 2 --micro-batch-size 32 --grad-accum 8 --steps 4 --warmup 2"
for S in s0 s1; do
  if [ $S = s0 ]; then SA="--num-layers 13 --emulate-first-stage"; else SA="--num-layers 11 --emulate-last-stage"; fi
  SMDT_LINK_STANDIN=relay SMDT_RING_GEMM_TN=1 run ${S}_base 400 python bench.py $SA $ST
  SMDT_LINK_STANDIN=relay SMDT_RING_GEMM_TN=1 SMDT_W_FILL=1 run ${S}_fill 400 python bench.py $SA $ST
  SMDT_LINK_STANDIN=relay SMDT_W_FILL=1 run ${S}_fill_blaslt 400 python bench.py $SA $ST
  SMDT_W_FILL=1 run ${S}_fill_copy 400 python bench.py $SA $ST
  run ${S}_copy 400 python bench.py $SA $ST
done
echo DONE
