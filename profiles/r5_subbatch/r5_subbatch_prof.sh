set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r5_subbatch_prof; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
ST="--num-layers 13 --emulate-first-stage --emulate-tp 2 --micro-batch-size 32 --grad-accum 8 --steps 2 --warmup 1 --comm-stats 0"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/def -o run --output-format csv -- python3 $R/bench.py $ST > $O/def.log 2>&1 && echo def ok &&
SMDT_SP_SUBBATCH=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/sub -o run --output-format csv -- python3 $R/bench.py $ST > $O/sub.log 2>&1 && echo sub ok
find $O -name '*kernel_trace.csv' -delete
