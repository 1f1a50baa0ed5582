#!/bin/bash
# Round 4: sequence-parallel norms writing into their all-gather slots (no ag_ring local copy):
# GPU equivalence test, LN kernel tests, then the emulated N = 8 stage ranks re-measured (A/B
# against the copying path in the same call via a patched spec) and the 1-GPU bench.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4r
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 2 "$R/$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step tests 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_parallel_gpu.py tests/test_kernels_gpu.py -k "gather or layernorm or norm or wgrad"
N8="--emulate-tp 2 --micro-batch-size 32 --grad-accum 8 --steps 6 --warmup 3"
step stage1_slots 300 python bench.py $N8 --num-layers 11 --emulate-last-stage
SMDT_SP_GATHER_SLOTS=0 step stage1_copy 300 python bench.py $N8 --num-layers 11 --emulate-last-stage
step stage0_slots 300 python bench.py $N8 --num-layers 13 --emulate-first-stage
SMDT_SP_GATHER_SLOTS=0 step stage0_copy 300 python bench.py $N8 --num-layers 13 --emulate-first-stage
step bench 300 python bench.py --steps 20 --warmup 5
echo DONE
