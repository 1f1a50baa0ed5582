# Tune the GEMM shapes missing from the committed TunableOp table (bench.py --tunableop 3) for the
# N = 1 step and the emulated N = 8 stage ranks, merge them on the box, then A/B the benches on the
# merged table against the committed one.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=gpurun_out/r5_tune; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
T=profiles/tunableop/gfx950_gpt345m_results.csv
ST="--num-layers 11 --emulate-last-stage --emulate-tp 2 --micro-batch-size 32 --grad-accum 8"
SF="--num-layers 13 --emulate-first-stage --emulate-tp 2 --micro-batch-size 32 --grad-accum 8"
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; grep -h '"metric"' $O/$n.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
run base_n1 300 python bench.py --steps 10 --warmup 3
run base_st 300 python bench.py --steps 4 --warmup 2 $ST
run tune_n1 600 python bench.py --steps 1 --warmup 2 --tunableop 3 --tune-out $O/tuned_n1.csv
run tune_st 600 python bench.py --steps 1 --warmup 2 --tunableop 3 --tune-out $O/tuned_st.csv $ST
run tune_sf 600 python bench.py --steps 1 --warmup 2 --tunableop 3 --tune-out $O/tuned_sf.csv $SF; touch $O/tuned_sf.csv
cp $T $O/committed.csv
python scripts/merge_tunableop.py $O/merged.csv $T $O/tuned_n1.csv $O/tuned_st.csv $O/tuned_sf.csv
cp $O/merged.csv $T
run new_n1 300 python bench.py --steps 10 --warmup 3
run new_st 300 python bench.py --steps 4 --warmup 2 $ST
cp $O/committed.csv $T
run base_n1b 300 python bench.py --steps 10 --warmup 3
cp $O/merged.csv $T
run new_n1b 300 python bench.py --steps 10 --warmup 3
echo DONE
