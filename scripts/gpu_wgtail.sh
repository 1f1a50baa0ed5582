#!/bin/bash
# wgrad tail split: wgrad GPU tests, then the default bench with the split on and off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/wgtail
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_parallel_gpu.py tests/test_kernels_gpu.py -k "wgrad" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py > $O/bench_on.log 2>&1 || { tail -20 $O/bench_on.log; exit 1; }
SMDT_WGRAD_TAIL_SPLIT=0 timeout -k 10 300 python -u bench.py > $O/bench_off.log 2>&1 || { tail -20 $O/bench_off.log; exit 1; }
timeout -k 10 300 python -u bench.py > $O/bench_on2.log 2>&1 || { tail -20 $O/bench_on2.log; exit 1; }
for f in bench_on bench_off bench_on2; do tail -1 $O/$f.log | cut -c1-190; done
