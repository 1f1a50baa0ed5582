#!/bin/bash
# A/B the flash-attention builds in build/variants/*.so on the GPT-2 345M attention shape
# (fwd + bwd, causal, with and without dropout). Runs on the GPU box.
set -u
mkdir -p gpurun_out
cp smdt_amd/_C.so /tmp/_C_orig.so
for v in build/variants/_C_*.so; do
  cp "$v" smdt_amd/_C.so
  for dp in 0 0.1; do
    timeout -k 10 120 python benchmarks/bench_attention.py --dropout $dp --sdpa 0 > /tmp/ab.json 2>/dev/null
    rc=$?
    [ $rc -ne 0 ] && { echo "ABORT $v rc=$rc"; cp /tmp/_C_orig.so smdt_amd/_C.so; exit $rc; }
    echo "$(basename $v) $(cat /tmp/ab.json)" | tee -a gpurun_out/ab_attention.log
  done
done
cp /tmp/_C_orig.so smdt_amd/_C.so
