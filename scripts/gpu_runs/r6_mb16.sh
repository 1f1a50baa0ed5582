# round 6: why the emulated tp2 stage 0 at 16 x 16 micro-batches runs 408 ms (kernel stats)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r6_mb16; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 SMDT_LINK_STANDIN=relay
N16="--emulate-tp 2 --micro-batch-size 16 --grad-accum 16 --num-layers 13 --emulate-first-stage --steps 2 --warmup 2 --comm-stats 0 --phase-probe 0"
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py $N16 > $O/prof.log 2>&1
rc=$?; cd $R; f=$(find $O/prof -name '*kernel_stats.csv' | head -n 1); cut -d, -f1-4 "$f" | head -n 25 | cut -c1-200; find $O/prof -name '*kernel_trace.csv' -delete; tail -n 1 $O/prof.log | cut -c1-200; exit $rc
