#!/bin/bash
# A/B of build/variants/_C_*.so on the bench attention shape (B32 S1024 H16 D64, dropout 0.1),
# then the default bench on the base build.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/ab2
cp smdt_amd/_C.so /tmp/_C_orig.so
for rep in 1 2; do
for v in build/variants/_C_*.so; do
  cp "$v" smdt_amd/_C.so
  timeout -k 10 120 python benchmarks/bench_attention.py --b ${ATTN_B:-32} --dropout 0.1 --sdpa 0 > /tmp/ab.json 2>/dev/null
  rc=$?
  [ $rc -ne 0 ] && { echo "ABORT $v rc=$rc"; cp /tmp/_C_orig.so smdt_amd/_C.so; exit $rc; }
  echo "$(basename $v) $(tail -1 /tmp/ab.json)" | tee -a gpurun_out/ab2/ab_attention.log
done
done
cp /tmp/_C_orig.so smdt_amd/_C.so
[ "${AB_BENCH:-1}" = 1 ] || exit 0
timeout -k 10 300 python -u bench.py > gpurun_out/ab2/bench.log 2>&1 || { tail -20 gpurun_out/ab2/bench.log; exit 1; }
tail -1 gpurun_out/ab2/bench.log | cut -c1-200
