# Which MIOpen state makes a fresh process fast: the user find / perf db (text) or the compiled
# kernel cache? ResNet-50 224 bf16 channels-last, 64 img, one GPU, no prewarm child in the timed runs.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r5_miopen; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
V="python benchmarks/bench_vision.py --model resnet50 --size 224 --batch 64 --steps 20 --warmup 5 --miopen-prewarm 0"
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; grep -h '"metric"' $O/$n.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
# 1. fresh: empty user db, empty kernel cache
MIOPEN_USER_DB_PATH=$O/udb_fresh MIOPEN_CUSTOM_CACHE_DIR=$O/kc_fresh run fresh 600 $V
# 2. populate a db + cache pair with a first process, then a second process on both
MIOPEN_USER_DB_PATH=$O/udb MIOPEN_CUSTOM_CACHE_DIR=$O/kc run populate 600 $V
MIOPEN_USER_DB_PATH=$O/udb MIOPEN_CUSTOM_CACHE_DIR=$O/kc run both 600 $V
# 3. the populated user db with an EMPTY kernel cache
MIOPEN_USER_DB_PATH=$O/udb MIOPEN_CUSTOM_CACHE_DIR=$O/kc_empty run db_only 600 $V
# 4. the kernel cache with an empty user db
MIOPEN_USER_DB_PATH=$O/udb_empty MIOPEN_CUSTOM_CACHE_DIR=$O/kc run cache_only 600 $V
ls -laR $O/udb $O/kc | head -40
du -sh $O/udb $O/kc
rm -rf $O/kc $O/kc_fresh $O/kc_empty
echo DONE
