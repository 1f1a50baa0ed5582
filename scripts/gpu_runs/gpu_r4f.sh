#!/bin/bash
# Round 4: GPU tests (smddp multi-bucket + sync-checked phases, flash dK/dV rework, wgrad BIAS
# template); bench A/B of the grouped-wgrad bias column sums (SMDT_WGRAD_BIAS=0) with a kernel
# trace of each arm; ResNet-50 vision bench with and without the framework's DDP wrapper and
# MIOpen's solver log (this round's vision runs picked MIOpen's naive kernels).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4f
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
step attn 120 python benchmarks/bench_attention.py --b 64 --sdpa 0 --dropout 0.1
step bench 300 python bench.py --steps 20 --warmup 5
SMDT_WGRAD_BIAS=0 step bench_nobias 300 python bench.py --steps 20 --warmup 5
cd /tmp
step prof_bench 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_bench" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 8 --warmup 3
SMDT_WGRAD_BIAS=0 step prof_bench_nobias 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_bench_nobias" -o run \
  --output-format csv -- python3 "$R/bench.py" --steps 8 --warmup 3
cd "$R"
step vision_r50_noddp 400 python benchmarks/bench_vision.py --model resnet50 --size 224 --batch 64 --steps 10 --warmup 3 --ddp none
step vision_r50 400 python benchmarks/bench_vision.py --model resnet50 --size 224 --batch 64 --steps 10 --warmup 3
MIOPEN_LOG_LEVEL=5 timeout -k 10 400 python benchmarks/bench_vision.py --model resnet50 --size 224 --batch 64 --steps 2 \
  --warmup 1 --ddp none 2>&1 | grep -E "Solver|solver|algo|Naive|naive|Find|Error|error|Warn|json|img" | sort | uniq -c | sort -rn | head -80 > $O/miopen_log_summary.txt
echo "miopen log rc=$?"
echo DONE
