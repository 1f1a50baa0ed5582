#!/bin/bash
# Round 4: GPU tests after the grouped-wgrad bias fix (MFMA-with-ones column sums, BIAS template),
# the smddp test's multi-bucket model and the dropout keep words (forward -> dQ kernel); attention
# microbench and the 1-GPU bench, each A/B against SMDT_FA_KEEP_WORDS=0 (re-hash); kernel trace of
# the bench; MIOpen probe of the ResNet-50 convolutions (the vision bench ran MIOpen's naive
# kernels this round).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4e
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
SMDT_FA_KEEP_WORDS=0 step attn_rehash 120 python benchmarks/bench_attention.py --b 64 --sdpa 0 --dropout 0.1
step bench 300 python bench.py --steps 20 --warmup 5
SMDT_FA_KEEP_WORDS=0 step bench_rehash 300 python bench.py --steps 20 --warmup 5
cd /tmp
step prof_bench 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_bench" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 8 --warmup 3
cd "$R"
step miopen_nhwc_bf16 300 python benchmarks/miopen_probe.py
MIOPEN_LOG_LEVEL=5 step miopen_nhwc_bf16_log 300 python benchmarks/miopen_probe.py
step miopen_nchw_bf16 300 python benchmarks/miopen_probe.py --nchw
step miopen_nhwc_fp32 300 python benchmarks/miopen_probe.py --fp32
echo DONE
