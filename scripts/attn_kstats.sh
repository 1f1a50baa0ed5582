#!/bin/bash
# Per-kernel times of the flash-attention kernels (rocprofv3 --kernel-trace --stats), no dropout
# and dropout 0.1, on the GPT-2 345M attention shape. GPU box only.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/attn_ks
cd /tmp && export TMPDIR=/tmp
for dp in 0 0.1; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/attn_ks/d$dp -o run --output-format csv -- \
    python3 $R/benchmarks/bench_attention.py --sdpa 0 --b 32 --h 16 --s 1024 --d 64 --dropout $dp > $R/gpurun_out/attn_ks/d$dp.log 2>&1
  rc=$?
  [ $rc -ne 0 ] && { echo "rc=$rc"; exit $rc; }
  tail -1 $R/gpurun_out/attn_ks/d$dp.log
  python3 $R/scripts/kstats.py $(ls $R/gpurun_out/attn_ks/d$dp/*kernel_stats.csv | head -1) | head -8
done
