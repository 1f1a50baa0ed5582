#!/bin/bash
# Round 4: the dK / dV kernel rework (row-constant term rows, per-slot LDS objects, buffer_load
# ... lds) checked and timed; the 1-GPU bench A/B of the grouped-wgrad bias column sums
# (SMDT_WGRAD_BIAS=0 = round-3 bias path) against the round-3 160.6 ms; a kernel trace of the
# bench; ResNet-50 with a private MIOpen database / kernel cache (round-4 opening run picked
# MIOpen's naive convolutions).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4d
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 6 "$R/$O/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
echo "HOME=$HOME user=$(id -un)"; ls -ld "$HOME" "$HOME/.config" "$HOME/.cache" 2>&1 | head -5
env | grep -i miopen || true
step tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_xgmi.py -k "flash or wgrad or smddp or tp_direct"
step attn 120 python benchmarks/bench_attention.py --b 64 --sdpa 0 --dropout 0.1
step bench 300 python bench.py --steps 20 --warmup 5
SMDT_WGRAD_BIAS=0 step bench_nobias 300 python bench.py --steps 20 --warmup 5
cd /tmp
step prof_bench 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_bench" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 8 --warmup 3
cd "$R"
MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache \
  step vision_r50 400 python benchmarks/bench_vision.py --model resnet50 --size 224 --batch 64 --steps 20 --warmup 5
echo DONE
