# Flash-attention A/B on one MI355X: the in-tree kernels vs benchmarks/bin/ab_ref_C.so (the same
# sources before the change), interleaved, at the bench shape; per-kernel stats of both.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=$R/gpurun_out/${OUT:-r5_attn_ab}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc; }
[ "${TESTS:-1}" = "1" ] && run tests 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "flash or attention"
A="--b 64 --sdpa 0 --dropout 0.1"
for i in $(seq 1 ${ROUNDS:-3}); do
  run ref_$i 150 python benchmarks/bench_attention.py $A --ext benchmarks/bin/ab_ref_C.so
  run new_$i 150 python benchmarks/bench_attention.py $A
  # optional third arm: the new build under extra environment (e.g. NEW_ENV2=SMDT_FA_DKDV_OCC=2)
  if [ -n "${NEW_ENV2:-}" ]; then run new2_$i 150 env $NEW_ENV2 python benchmarks/bench_attention.py $A; fi
done
cd /tmp
run prof_new 200 rocprofv3 --kernel-trace --stats -d "$O/prof_new" -o run --output-format csv -- python3 "$R/benchmarks/bench_attention.py" $A
run prof_ref 200 rocprofv3 --kernel-trace --stats -d "$O/prof_ref" -o run --output-format csv -- python3 "$R/benchmarks/bench_attention.py" $A --ext "$R/benchmarks/bin/ab_ref_C.so"
cd "$R"
find $O -name '*kernel_trace.csv' -delete
[ "${BENCH:-1}" = "1" ] && run bench 300 python bench.py --steps 20 --warmup 5
echo DONE
