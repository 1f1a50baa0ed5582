#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/abf
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 > gpurun_out/abf/$n.log 2>&1 || { tail -20 gpurun_out/abf/$n.log; exit 1; }
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abf/$n.log)"
}
run base SMDT_FUSED_FC1=0
run fused SMDT_FUSED_FC1=1
run base2 SMDT_FUSED_FC1=0
run fused2 SMDT_FUSED_FC1=1
