#!/bin/bash
# Round-4 opening GPU session: GPU tests, the 1-GPU bench, flash-attention PMC counters at the
# bench's shape (B64 S1024 H16 D64, dropout 0.1) and kernel traces of the vision configs.
# Stops at the first step that faults / aborts / times out (exit status not in {0,1}).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
mkdir -p gpurun_out/r4a
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/gpurun_out/r4a/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 8 "$R/gpurun_out/r4a/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
step bench 300 python bench.py --steps 20 --warmup 5
step attn 120 python benchmarks/bench_attention.py --b 64 --sdpa 0 --dropout 0.1
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU"
P2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_VALU_MFMA_COEXEC_CYCLES"
cd /tmp
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  step pmc_attn_p$i 120 rocprofv3 --pmc $P --kernel-trace -d "$R/gpurun_out/r4a/pmc/p$i" -o run --output-format csv -- \
    python3 "$R/benchmarks/bench_attention.py" --b 64 --sdpa 0 --dropout 0.1
done
cd "$R"
step vision_r50 300 python benchmarks/bench_vision.py --model resnet50 --size 224 --batch 64 --steps 20 --warmup 5
step vision_swin 300 python benchmarks/bench_vision.py --model swin_b --size 128 --batch 40 --steps 20 --warmup 5
cd /tmp
step prof_r50 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r4a/prof_r50" -o run --output-format csv -- \
  python3 "$R/benchmarks/bench_vision.py" --model resnet50 --size 224 --batch 64 --steps 5 --warmup 3
step prof_swin 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r4a/prof_swin" -o run --output-format csv -- \
  python3 "$R/benchmarks/bench_vision.py" --model swin_b --size 128 --batch 40 --steps 5 --warmup 3
P3="SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT"
cd /tmp
step pmc_attn_p3 120 rocprofv3 --pmc $P3 --kernel-trace -d "$R/gpurun_out/r4a/pmc/p3" -o run --output-format csv -- \
  python3 "$R/benchmarks/bench_attention.py" --b 64 --sdpa 0 --dropout 0.1
echo DONE
