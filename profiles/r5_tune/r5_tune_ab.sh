set -u
O=gpurun_out/r5_tune_ab; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
T=profiles/tunableop/gfx950_gpt345m_results.csv
ST="--num-layers 11 --emulate-last-stage --emulate-tp 2 --micro-batch-size 32 --grad-accum 8"
cp $T $O/new.csv; git_old=$O/old.csv
grep -v "tn_1024_65536_50304_ld\|tn_1024_16384_25216_ld\|tn_25216_16384_1024_ld" $T > $O/old.csv
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; grep -h '"metric"' $O/$n.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
for i in 1 2; do
cp $O/old.csv $T; run old_n1_$i 300 python bench.py --steps 10 --warmup 3
cp $O/new.csv $T; run new_n1_$i 300 python bench.py --steps 10 --warmup 3
cp $O/old.csv $T; run old_st_$i 300 python bench.py --steps 4 --warmup 2 $ST
cp $O/new.csv $T; run new_st_$i 300 python bench.py --steps 4 --warmup 2 $ST
done
echo DONE
