#!/bin/bash
# Round 4: 2-D SwiGLU kernels (no 64-bit div / mod per chunk) vs the grid-stride ones
# (SMDT_SWIGLU_2D=0), tests, then the SFT emulated DP8 rank with the 2-D form.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4au
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 1 "$R/$O/$name.log" | cut -c1-330
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_hf_models.py
step ew_2d 150 python benchmarks/bench_elementwise.py
SMDT_SWIGLU_2D=0 step ew_gs 150 python benchmarks/bench_elementwise.py
step ew_2d2 150 python benchmarks/bench_elementwise.py
SMDT_SWIGLU_2D=0 step ew_gs2 150 python benchmarks/bench_elementwise.py
echo DONE
