#!/bin/bash
# Round 4: grouped-wgrad bias cost in isolation (benchmarks/bench_wgrad_bias.py: no bias / QKV+fc1
# bias tiles / bias on every problem, 5 GPT-2 layers at 65,536 tokens) and a PMC pass over it.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4m
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 3 "$R/$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step wgrad_bias 180 python benchmarks/bench_wgrad_bias.py --layers 5
step wgrad_bias2 180 python benchmarks/bench_wgrad_bias.py --layers 5
step wgrad_bias_1layer 180 python benchmarks/bench_wgrad_bias.py --layers 1
echo DONE
