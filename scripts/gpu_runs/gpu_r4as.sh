#!/bin/bash
# Round 4: fused Adam as one batch of U float4 vectors per thread vs the grid-stride form.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4as
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "adam or optim" > $O/tests.log 2>&1 || { tail -5 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for u in 0 1 2 4 0 2 4; do
  SMDT_ADAM_U=$u timeout -k 10 120 python benchmarks/bench_adam.py >> $O/adam.log 2>&1 || exit $?
done
grep '^{' $O/adam.log
