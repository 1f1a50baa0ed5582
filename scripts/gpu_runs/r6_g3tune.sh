# round 6: TunableOp winners for the GPT-3 6.7B tp4 stage shapes (tuned once, then the stage with
# the tuned table vs the library heuristics, alternated)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r6_g3tune; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-140; [ $rc -eq 0 ] || exit $rc; }
G="--emulate-tp 4 --hidden-size 4096 --num-attention-heads 32 --seq-length 2048 --micro-batch-size 4 --grad-accum 8 --num-layers 16"
run tune0 900 python bench.py $G --emulate-first-stage --steps 1 --warmup 1 --tunableop 2 --tune-out $O/g3_tuned_s0.csv --tune-ms 30
run tune1 900 python bench.py $G --emulate-last-stage --steps 1 --warmup 1 --tunableop 2 --tune-out $O/g3_tuned_s1.csv --tune-ms 30
python scripts/merge_tunableop.py $O/g3_tuned.csv $O/g3_tuned_s0.csv $O/g3_tuned_s1.csv > $O/merge.log 2>&1 || cp $O/g3_tuned_s0.csv $O/g3_tuned.csv
for i in 1 2; do
SMDT_TUNED_GEMMS=$O/g3_tuned.csv run s0_tuned_$i 500 python bench.py $G --emulate-first-stage --steps 3 --warmup 2 --tunableop 1
run s0_heur_$i 500 python bench.py $G --emulate-first-stage --steps 3 --warmup 2 --tunableop 0
done
echo DONE
