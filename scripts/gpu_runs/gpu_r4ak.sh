#!/bin/bash
# Round 4: after removing the neutral straight-line dQ / dK-dV variants — kernel tests, attention
# microbench, bench.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4ak
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
step tests 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests
step attn 120 python benchmarks/bench_attention.py --b 64 --sdpa 0 --dropout 0.1
step bench 300 python bench.py --steps 20 --warmup 5
echo DONE
