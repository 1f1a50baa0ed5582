#!/bin/bash
# Round 4 final check on one MI355X: GPU suite, smoke, headline bench twice, attention at the
# step shape, GPT-2 small like-for-like (NB3's mbs 12 x GA 4), vision configs, and a kernel trace
# of the headline step.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4_final
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
step pytest_gpu 700 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests
step smoke 180 python __graft_entry__.py smoke
step bench 300 python bench.py --steps 20 --warmup 5
step bench2 300 python bench.py --steps 20 --warmup 5
step attn 120 python benchmarks/bench_attention.py --b 64 --sdpa 0 --dropout 0.1
step gpt2_small 300 python bench.py --num-layers 12 --hidden-size 768 --num-attention-heads 12 --micro-batch-size 12 --grad-accum 4 --steps 10 --warmup 3
step vision_r50 500 python benchmarks/bench_vision.py --model resnet50 --size 224 --batch 64 --steps 20 --warmup 5
step vision_swin 500 python benchmarks/bench_vision.py --model swin_b --size 128 --batch 40 --steps 20 --warmup 5
cd /tmp
step prof 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 3 --warmup 3
cd "$R"
f=$(find "$O/prof" -name '*kernel_trace.csv' | head -n 1)
python scripts/ktrace_steps.py "$f" 40 > "$O/last_step_breakdown.txt" && head -n 14 "$O/last_step_breakdown.txt"
find "$O/prof" -name '*kernel_trace.csv' -delete
echo DONE
