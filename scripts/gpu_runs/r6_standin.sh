# round 6: emulated tp2pp2 stage ranks under the paced link stand-in (SMDT_LINK_STANDIN=relay:
# the relay's modelled 256 GB/s and its 64 workgroups on the side stream), plain vs the sub-batch
# interleave (SMDT_SP_SUBBATCH=2), against the in-line-copy emulation
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/${OUT:-r6_standin}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
run tests 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_kernels_gpu.py::test_paced_copy_copies_and_holds_for_its_link_time tests/test_relay.py
ST="--emulate-tp 2 --micro-batch-size 32 --grad-accum 8 --steps 4 --warmup 2"
for S in s0 s1; do
  if [ $S = s0 ]; then SA="--num-layers 13 --emulate-first-stage"; else SA="--num-layers 11 --emulate-last-stage"; fi
  run ${S}_copy 400 python bench.py $SA $ST
  SMDT_LINK_STANDIN=relay run ${S}_relay 400 python bench.py $SA $ST
  SMDT_LINK_STANDIN=relay SMDT_SP_SUBBATCH=2 run ${S}_relay_sub 400 python bench.py $SA $ST
done
echo DONE
