#!/bin/bash
# Start-of-session check: full GPU suite, smoke, default bench, kernel-trace step profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${SANITY_OUT:-r3_sanity}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
f=$(ls $O/prof/*/run_kernel_trace.csv $O/prof/run_kernel_trace.csv 2>/dev/null | head -n 1)
python3 scripts/ktrace_steps.py "$f" > $O/last_step_breakdown.txt 2>&1
head -n 40 $O/last_step_breakdown.txt
