#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/abw
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 > gpurun_out/abw/$n.log 2>&1 || { tail -20 gpurun_out/abw/$n.log; exit 1; }
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abw/$n.log)"
}
run grouped SMDT_DEFER_WGRAD=1
run blaslt SMDT_DEFER_WGRAD=0 SMDT_WGRAD_IMPL=blaslt
run auto SMDT_DEFER_WGRAD=0 SMDT_WGRAD_IMPL=auto
run grouped2 SMDT_DEFER_WGRAD=1
