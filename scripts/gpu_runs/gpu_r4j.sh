#!/bin/bash
# Round 4: vision configs with the augmentation HIP kernels + prefetcher (swin_b 128 and ResNet-50
# 224, each after bench_vision's MIOpen prewarm child) and their kernel traces; the per-rank
# emulation + schedule prediction again, the emulated stages now issuing each micro-batch's W
# GEMMs as one group after its backward (as a zero-bubble stage does).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4j
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 3 "$R/$O/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step vision_r50 500 python benchmarks/bench_vision.py --model resnet50 --size 224 --batch 64 --steps 20 --warmup 5
step vision_swin 500 python benchmarks/bench_vision.py --model swin_b --size 128 --batch 40 --steps 20 --warmup 5
cd /tmp
step prof_r50 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_r50" -o run --output-format csv -- \
  python3 "$R/benchmarks/bench_vision.py" --model resnet50 --size 224 --batch 64 --steps 8 --warmup 3 --miopen-prewarm 0
step prof_swin 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_swin" -o run --output-format csv -- \
  python3 "$R/benchmarks/bench_vision.py" --model swin_b --size 128 --batch 40 --steps 8 --warmup 3 --miopen-prewarm 0
cd "$R"
step predict 900 python -u benchmarks/predict_scaling.py --out $O/predict
echo DONE
