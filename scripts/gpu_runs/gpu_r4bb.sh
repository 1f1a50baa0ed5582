#!/bin/bash
# Round 4: LM-head GEMM + CE as one op (ce_fused) — CE / model GPU tests, kernel time, bench A/B
# against the separate ce_stats / ce_bwd path (SMDT_LM_HEAD_CE=0), interleaved.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/${R4BB_OUT:-r4bb}
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 1 "$R/$O/$name.log" | cut -c1-420
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step tests 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "lm_head or cross"
step model_tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_model_gpu.py
for r in a b; do
  export SMDT_LM_HEAD_CE=1; step bench_fused_$r 300 python bench.py --steps 20 --warmup 5
  export SMDT_LM_HEAD_CE=0; step bench_sep_$r 300 python bench.py --steps 20 --warmup 5
done
export SMDT_LM_HEAD_CE=1
cd /tmp
step prof 400 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv -- python "$R/bench.py" --steps 3 --warmup 2
echo DONE
