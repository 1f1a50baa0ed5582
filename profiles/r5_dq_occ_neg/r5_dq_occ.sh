# dQ kernel at 4 workgroups per CU (2 K / V stage slots, 128 VGPRs) vs the default 2 x 3 slots:
# benchmarks/bin/ab_var_C.so built with SMDT_KERNEL_FLAGS="flash_attn.hip:-DSMDT_FA_DQ_OCC=4,
# -DSMDT_FA_DQ_BUF=2", interleaved with the in-tree build at the bench shape.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r5_dq_occ; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
A="--b 64 --sdpa 0 --dropout 0.1"
for i in 1 2 3; do
  run def_$i 150 python benchmarks/bench_attention.py $A
  run var_$i 150 python benchmarks/bench_attention.py $A --ext benchmarks/bin/ab_var_C.so
done
cd /tmp
run prof_var 200 rocprofv3 --kernel-trace --stats -d "$O/prof_var" -o run --output-format csv -- python3 "$R/benchmarks/bench_attention.py" $A --ext "$R/benchmarks/bin/ab_var_C.so"
run prof_def 200 rocprofv3 --kernel-trace --stats -d "$O/prof_def" -o run --output-format csv -- python3 "$R/benchmarks/bench_attention.py" $A
find $O -name '*kernel_trace.csv' -delete
echo DONE
