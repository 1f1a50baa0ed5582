#!/bin/bash
# dQ beside dK/dV on a side stream: attention tests, attention A/B, bench A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/faov
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "flash or attention or gpt" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for ov in 1 0; do
    SMDT_FA_BWD_OVERLAP=$ov timeout -k 10 120 python benchmarks/bench_attention.py --b 64 --dropout 0.1 --sdpa 0 > /tmp/a.json 2>/dev/null || exit 1
    echo "overlap=$ov $(tail -1 /tmp/a.json)" | tee -a $O/ab.log | cut -c1-160
  done
done
timeout -k 10 300 python -u bench.py > $O/bench_on.log 2>&1 || { tail -20 $O/bench_on.log; exit 1; }
SMDT_FA_BWD_OVERLAP=0 timeout -k 10 300 python -u bench.py > $O/bench_off.log 2>&1 || { tail -20 $O/bench_off.log; exit 1; }
for f in bench_on bench_off; do tail -1 $O/$f.log | cut -c1-170; done
