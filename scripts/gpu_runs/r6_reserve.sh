# round 6: paced relay stand-in, stage ranks: CU reservation for in-flight exchanges (gemm_tn chunk
# grids sized to the CUs the exchange leaves) and ring-chunk GEMMs on gemm_tn, A/B in one call
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/${OUT:-r6_reserve}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 SMDT_LINK_STANDIN=relay
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
ST="--emulate-tp 2 --micro-batch-size 32 --grad-accum 8 --steps 4 --warmup 2"
SA="--num-layers 13 --emulate-first-stage"
SMDT_EXCHANGE_CU_RESERVE=0 run s0_noreserve 400 python bench.py $SA $ST
run s0_reserve 400 python bench.py $SA $ST
SMDT_RING_GEMM_TN=1 run s0_reserve_tn 400 python bench.py $SA $ST
SMDT_FUSED_BIAS_GELU=0 SMDT_EXCHANGE_CU_RESERVE=0 run s0_blaslt 400 python bench.py $SA $ST
SMDT_LINK_STANDIN=256:16 SMDT_EXCHANGE_CU_RESERVE=0 run s0_16wg 400 python bench.py $SA $ST
SMDT_LINK_STANDIN=256:16 run s0_16wg_reserve 400 python bench.py $SA $ST
SMDT_LINK_STANDIN=relay SMDT_RING_GEMM_TN=1 SMDT_SP_SUBBATCH=2 run s0_sub_tn 400 python bench.py $SA $ST
echo DONE
