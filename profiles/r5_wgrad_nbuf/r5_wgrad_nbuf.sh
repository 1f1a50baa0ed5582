# Grouped wgrad: 4- vs 5-buffer LDS-DMA stage ring (SMDT_WGRAD_NBUF), microbenchmark + step A/B,
# and the wgrad GPU tests on the 5-buffer kernel.
set -u
O=gpurun_out/r5_wgrad_nbuf; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
SMDT_WGRAD_NBUF=5 run tests5 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k wgrad
for i in 1 2; do
  SMDT_WGRAD_NBUF=4 run micro4_$i 200 python benchmarks/bench_wgrad_bias.py
  SMDT_WGRAD_NBUF=5 run micro5_$i 200 python benchmarks/bench_wgrad_bias.py
done
for i in 1 2; do
  SMDT_WGRAD_NBUF=4 run bench4_$i 300 python bench.py --steps 15 --warmup 3
  SMDT_WGRAD_NBUF=5 run bench5_$i 300 python bench.py --steps 15 --warmup 3
done
echo DONE
