#!/bin/bash
# Round 4 end-of-round check on the committed tree: the whole GPU suite, smoke(), the 1-GPU bench
# twice, and a rocprofv3 kernel-stats profile of the bench step.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/${R4AZ_OUT:-r4az}
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 2 "$R/$O/$name.log" | cut -c1-420
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 300 python bench.py --steps 20 --warmup 5
step bench2 300 python bench.py --steps 20 --warmup 5
cd /tmp
step prof 400 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv -- python "$R/bench.py" --steps 3 --warmup 2
echo DONE
