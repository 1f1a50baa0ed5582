# round 6: W fillers third form (grouped launch per wait; optional filler stream) under the paced
# relay stand-in, stage 0 / 1, with the GPU filler tests
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/${OUT:-r6_fill3}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 SMDT_LINK_STANDIN=relay
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
run tests 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_parallel_gpu.py -k w_fillers
ST="--emulate-tp 2 --micro-batch-size 32 --grad-accum 8 --steps 4 --warmup 2"
for S in s0 s1; do
  if [ $S = s0 ]; then SA="--num-layers 13 --emulate-first-stage"; else SA="--num-layers 11 --emulate-last-stage"; fi
  run ${S}_grouped 400 python bench.py $SA $ST
  SMDT_W_FILL_STREAM=1 run ${S}_stream 400 python bench.py $SA $ST
  SMDT_W_FILL_STREAM=1 SMDT_W_FILL_US=250 run ${S}_stream250 400 python bench.py $SA $ST
  SMDT_W_FILL_STREAM=1 SMDT_W_FILL_US=500 run ${S}_stream500 400 python bench.py $SA $ST
done
echo DONE
