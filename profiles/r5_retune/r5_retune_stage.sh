# Re-tune (TunableOp, every candidate, longer per-shape budget) the GEMM shapes of the emulated
# N = 8 stage ranks in situ, then A/B the last-stage rank on the committed table vs the re-tuned one.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r5_retune; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
T=profiles/tunableop/gfx950_gpt345m_results.csv
ST="--num-layers 11 --emulate-last-stage --emulate-tp 2 --micro-batch-size 32 --grad-accum 8"
SF="--num-layers 13 --emulate-first-stage --emulate-tp 2 --micro-batch-size 32 --grad-accum 8"
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; grep -h '"metric"' $O/$n.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc; }
run tune_st 900 python bench.py --steps 1 --warmup 2 --tunableop 2 --tune-ms 150 --tune-out $O/retuned_st.csv $ST
run tune_sf 900 python bench.py --steps 1 --warmup 2 --tunableop 2 --tune-ms 150 --tune-out $O/retuned_sf.csv $SF
cp $T $O/committed.csv
python scripts/merge_tunableop.py $O/merged.csv $T $O/retuned_st.csv $O/retuned_sf.csv
for i in 1 2; do
  cp $O/committed.csv $T; run old_st_$i 300 python bench.py --steps 4 --warmup 2 $ST
  cp $O/merged.csv $T; run new_st_$i 300 python bench.py --steps 4 --warmup 2 $ST
  cp $O/committed.csv $T; run old_sf_$i 300 python bench.py --steps 4 --warmup 2 $SF
  cp $O/merged.csv $T; run new_sf_$i 300 python bench.py --steps 4 --warmup 2 $SF
done
cp $O/committed.csv $T
echo DONE
