#!/bin/bash
# Round 4: GPU tests (smddp timing inside a stats step, augmentation kernels); bench with the
# grouped-wgrad bias fragment rotated to a compile-time index + kernel trace; vision: a separate
# warm-up process, then the next ResNet-50 process under a kernel trace (is the second process
# slow?) and a third; kernel trace of one emulated N = 8 rank (tp2pp2 last stage).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4i
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
step r50_p1 400 python benchmarks/bench_vision.py --model resnet50 --size 224 --batch 64 --steps 10 --warmup 3 --miopen-prewarm 0
cd /tmp
step r50_p2_prof 400 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_r50_p2" -o run --output-format csv -- \
  python3 "$R/benchmarks/bench_vision.py" --model resnet50 --size 224 --batch 64 --steps 10 --warmup 3 --miopen-prewarm 0
cd "$R"
step r50_p3 400 python benchmarks/bench_vision.py --model resnet50 --size 224 --batch 64 --steps 20 --warmup 5 --miopen-prewarm 0
cd /tmp
step prof_n8_stage1 400 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_n8_stage1" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 2 --warmup 2 --num-layers 11 --emulate-tp 2 --micro-batch-size 32 --grad-accum 8
cd "$R"
echo DONE
