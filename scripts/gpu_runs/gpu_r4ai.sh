#!/bin/bash
# Round 4: re-tune the headline step's GEMMs with a longer TunableOp budget per shape, merge into
# the preloaded table, and A/B the bench against the committed table in the same call.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4ai
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 2 "$R/$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step tune 600 python bench.py --tunableop 2 --tune-ms 400 --tune-out $R/$O/tuned_r%d.csv --steps 2 --warmup 2
python scripts/merge_tunableop.py $O/merged.csv profiles/tunableop/gfx950_gpt345m_results.csv $O/tuned_r0.csv
step bench_old 300 python bench.py --steps 20 --warmup 5
SMDT_TUNED_GEMMS=$R/$O/merged.csv step bench_new 300 python bench.py --steps 20 --warmup 5
step bench_old2 300 python bench.py --steps 20 --warmup 5
SMDT_TUNED_GEMMS=$R/$O/merged.csv step bench_new2 300 python bench.py --steps 20 --warmup 5
echo DONE
