# round 6: the QKV forward GEMM with bias, in the forms torch offers, with the bench's TunableOp table
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r6_qkv; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -u benchmarks/bench_qkv_bias.py > $O/bench.log 2>&1 && \
timeout -k 10 200 python -u benchmarks/bench_qkv_bias.py --tunableop 0 > $O/bench_notune.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/benchmarks/bench_qkv_bias.py --reps 5 > $O/prof.log 2>&1
rc=$?; cd $R; tail -n 1 $O/bench.log; tail -n 1 $O/bench_notune.log; f=$(find $O/prof -name '*kernel_stats.csv' | head -n 1); cut -d, -f1-4 "$f" | head -n 12; find $O/prof -name '*kernel_trace.csv' -delete; exit $rc
