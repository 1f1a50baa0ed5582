#!/bin/bash
# Round 4: GPU tests (smddp sync-checked step past the bucket rebuild, augment prefetcher); bench
# with the grouped-wgrad bias tiles re-reading their fragment (no branches) + kernel trace; vision
# (ResNet-50 224 / swin_b 128) with the MIOpen prewarm process and prefetched augmentation + kernel
# traces; the N = 4 rehearsal-stall isolation (Gloo CUDA reduce-scatter probe, traced rehearsal).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4g
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
step vision_r50_inline 300 python benchmarks/bench_vision.py --model resnet50 --size 224 --batch 64 --steps 20 --warmup 5 --prefetch 0 --miopen-prewarm 0
step vision_swin 500 python benchmarks/bench_vision.py --model swin_b --size 128 --batch 40 --steps 20 --warmup 5
cd /tmp
step prof_r50 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_r50" -o run --output-format csv -- \
  python3 "$R/benchmarks/bench_vision.py" --model resnet50 --size 224 --batch 64 --steps 8 --warmup 3 --miopen-prewarm 0
step prof_swin 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_swin" -o run --output-format csv -- \
  python3 "$R/benchmarks/bench_vision.py" --model swin_b --size 128 --batch 40 --steps 8 --warmup 3 --miopen-prewarm 0
cd "$R"
for n in 2 4; do
  echo "=== gloo_probe_n$n"
  timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29600 + n)) benchmarks/gloo_cuda_probe.py --buckets 75 --mb 16 --limit 90 > $O/gloo_probe_n$n.log 2>&1
  echo "rc=$?"; grep '^{' $O/gloo_probe_n$n.log || tail -5 $O/gloo_probe_n$n.log
done
echo "=== rehearse_n4"
SMDT_BENCH_BACKEND=gloo SMDT_COLLECTIVE_LOG=$R/$O/clog SMDT_BENCH_DUMP_AFTER=100 timeout -k 10 160 \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29611 \
  bench.py --gpus 4 --steps 2 --warmup 1 --tunableop 0 --seqs-per-gpu 8 > $O/rehearse_n4.log 2>&1
echo "rc=$?"; grep '^{' $O/rehearse_n4.log | cut -c1-300; wc -l $O/clog.rank* 2>/dev/null
echo DONE
