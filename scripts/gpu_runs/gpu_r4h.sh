#!/bin/bash
# Round 4: GPU tests; bench with the grouped-wgrad bias sums as VALU on the re-read fragment +
# kernel trace; vision with a 13-step MIOpen prewarm child and prefetched augmentation; then the
# per-rank emulation measurements + schedule simulation of benchmarks/predict_scaling.py
# (N = 8 tp2pp2dp2 + SP with zb / zbh1 / 1f1b / interleaved; GPT-3 6.7B TP4 PP2 + SP).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4h
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 4 "$R/$O/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread
step bench 300 python bench.py --steps 20 --warmup 5
cd /tmp
step prof_bench 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_bench" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 8 --warmup 3
cd "$R"
step vision_r50 500 python benchmarks/bench_vision.py --model resnet50 --size 224 --batch 64 --steps 20 --warmup 5
step vision_swin 500 python benchmarks/bench_vision.py --model swin_b --size 128 --batch 40 --steps 20 --warmup 5
step predict 900 python -u benchmarks/predict_scaling.py --out $O/predict
echo DONE
