# ln_partials_reduce / bias colsum with 8 load chains (new) vs 4 (benchmarks/bin/ab_ref_C.so):
# per-kernel stats on the emulated stage-1 rank and the N = 1 step, then the LN GPU tests.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r5_colsum; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
SO=$R/smdt_amd/_C.so
cp $SO $O/new_C.so
ST="--num-layers 11 --emulate-last-stage --emulate-tp 2 --micro-batch-size 32 --grad-accum 8 --steps 2 --warmup 1 --comm-stats 0"
cd /tmp
for v in new ref new2 ref2; do
  case $v in new*) cp $O/new_C.so $SO ;; ref*) cp $R/benchmarks/bin/ab_ref_C.so $SO ;; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/st_$v -o run --output-format csv -- python3 $R/bench.py $ST > $O/st_$v.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/n1_$v -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --comm-stats 0 > $O/n1_$v.log 2>&1 || exit 1
  echo "$v done"
done
cp $O/new_C.so $SO
cd $R
find $O -name '*kernel_trace.csv' -delete
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "norm or layernorm or bias" > $O/tests.log 2>&1; echo "tests rc=$?"; tail -1 $O/tests.log
