#!/bin/bash
# One GPU measurement batch (run via gpurun from the repo root): kernel numerics, the headline
# bench + a rocprofv3 kernel profile, like-for-like reference configs and the north-star 6.7B
# config on one GPU, and the hipBLASLt epilogue probe. Every step has its own time limit; the
# script stops at the first failure. Logs: gpurun_out/r1c/<step>.log
set -o pipefail
OUT=gpurun_out/r1c
mkdir -p "$OUT"
export TMPDIR=/tmp
( while sleep 45; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
step() {
  local name=$1 t=$2
  shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -4 "$OUT/$name.log"
  return $rc
}
ONLY=${ONLY:-kernels,bench,prof,gpt2small,swinb,resnet50,gpt3,probe}
want() { [[ ",$ONLY," == *",$1,"* ]]; }
if want kernels; then
  step kernels 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_parallel_gpu.py tests/test_xgmi.py -x -q \
    --timeout 120 --timeout-method thread || exit 1
fi
if want bench; then step bench 400 python -u bench.py --steps 20 --warmup 3 || exit 1; fi
if want prof; then
  step prof 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 2 || exit 1
fi
if want gpt2small; then
  step gpt2small 400 python -u bench.py --num-layers 12 --hidden-size 768 --num-attention-heads 12 \
    --micro-batch-size 12 --grad-accum 4 --steps 10 --warmup 3 || exit 1
fi
if want swinb; then step swinb 400 python -u benchmarks/bench_vision.py --model swin_b --size 128 --batch 40 || exit 1; fi
if want resnet50; then
  step resnet50 400 python -u benchmarks/bench_vision.py --model resnet50 --size 224 --batch 64 || exit 1
fi
if want gpt3; then
  step gpt3 700 python -u bench.py --num-layers 32 --hidden-size 4096 --num-attention-heads 32 --seq-length 2048 \
    --micro-batch-size 4 --steps 4 --warmup 2 || exit 1
fi
if want probe; then
  hipcc -O2 scripts/probe_blaslt_epilogue.cpp -lhipblaslt -o /tmp/probe_epi && step probe 120 /tmp/probe_epi
fi
