# Re-tune the N = 1 step's GEMM shapes in situ (TunableOp, 150 ms per shape), A/B against the
# committed table, interleaved.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r5_retune_n1; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
T=profiles/tunableop/gfx950_gpt345m_results.csv
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; grep -h '"metric"' $O/$n.log | cut -c1-150; [ $rc -eq 0 ] || exit $rc; }
run tune_n1 900 python bench.py --steps 1 --warmup 2 --tunableop 2 --tune-ms 150 --tune-out $O/retuned_n1.csv
cp $T $O/committed.csv
python scripts/merge_tunableop.py $O/merged.csv $T $O/retuned_n1.csv
for i in 1 2 3; do
  cp $O/committed.csv $T; run old_$i 300 python bench.py --steps 15 --warmup 3
  cp $O/merged.csv $T; run new_$i 300 python bench.py --steps 15 --warmup 3
done
cp $O/committed.csv $T
echo DONE
