# round 6: the xGMI engine's DDP / ZeRO collectives captured in a HIP graph (2 processes, 1 GPU)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r6_xgraph; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_xgmi.py -k "graph or cross_process" > $O/tests.log 2>&1
rc=$?; tail -n 15 $O/tests.log; exit $rc
