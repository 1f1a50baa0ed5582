#!/bin/bash
# Attention iteration: flash-attention GPU tests, microbench at the headline shape (with / without
# dropout), then the 1-GPU bench. Stops at the first step that faults / aborts / times out.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 12 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_attn 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q -m gpu -k "flash or attention or dropout or gpt" --timeout 120 --timeout-method thread
step attn_drop 120 python benchmarks/bench_attention.py --b 32 --h 16 --s 1024 --d 64 --dropout 0.1 --sdpa 0
step attn_nodrop 120 python benchmarks/bench_attention.py --b 32 --h 16 --s 1024 --d 64 --dropout 0 --sdpa 0
step bench 300 python bench.py --steps 10 --warmup 3
echo DONE
