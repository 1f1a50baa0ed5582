# round 6: 2-rank ring exchanges in row pieces (SMDT_RING_PIECES) under the paced relay stand-in
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/${OUT:-r6_pieces}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 SMDT_LINK_STANDIN=relay
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
run tests 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gemm_tn_gpu.py -k "sp_fused or ring_pieces"
ST="--emulate-tp 2 --micro-batch-size 32 --grad-accum 8 --steps 4 --warmup 2"
for S in s0 s1; do
  if [ $S = s0 ]; then SA="--num-layers 13 --emulate-first-stage"; else SA="--num-layers 11 --emulate-last-stage"; fi
  run ${S}_p1 400 python bench.py $SA $ST
  SMDT_RING_PIECES=2 run ${S}_p2 400 python bench.py $SA $ST
  SMDT_RING_PIECES=4 run ${S}_p4 400 python bench.py $SA $ST
done
SMDT_RING_PIECES=2 run s0_p2_copy 400 env SMDT_LINK_STANDIN=0 python bench.py --num-layers 13 --emulate-first-stage $ST
echo DONE
