# Generate the MIOpen user find / perf db (text) of the Oxford-Pet models on gfx950, then time a
# fresh process (empty kernel cache) with and without it, ResNet-50 and swin_b.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r5_miopen_seed; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
R50="python benchmarks/bench_vision.py --model resnet50 --size 224 --batch 64 --steps 20 --warmup 5 --miopen-prewarm 0"
SWIN="python benchmarks/bench_vision.py --model swin_b --size 128 --batch 40 --steps 20 --warmup 5 --miopen-prewarm 0"
run() { local n=$1 t=$2; shift 2; local t0=$(date +%s); echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc wall=$(( $(date +%s) - t0 ))s"; grep -h '"metric"' $O/$n.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
MIOPEN_USER_DB_PATH=$O/udb MIOPEN_CUSTOM_CACHE_DIR=$O/kc1 run gen_r50 600 $R50
MIOPEN_USER_DB_PATH=$O/udb MIOPEN_CUSTOM_CACHE_DIR=$O/kc1 run gen_swin 600 $SWIN
MIOPEN_USER_DB_PATH=$O/udb0 MIOPEN_CUSTOM_CACHE_DIR=$O/kc2 run swin_fresh 600 $SWIN
MIOPEN_USER_DB_PATH=$O/udb MIOPEN_CUSTOM_CACHE_DIR=$O/kc3 run swin_db 600 $SWIN
MIOPEN_USER_DB_PATH=$O/udb MIOPEN_CUSTOM_CACHE_DIR=$O/kc4 run r50_db 600 $R50
ls -la $O/udb; rm -rf $O/kc1 $O/kc2 $O/kc3 $O/kc4
echo DONE
