# round 6: fc1 bias+GeLU / fc2 dgrad+GeLU' GEMMs at the N = 1 bench shape: gemm_tn epilogues vs
# hipBLASLt's own GELU_AUX_BIAS / DGELU epilogues vs library GEMM + elementwise
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r6_gelu; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
true && \
timeout -k 10 300 python -u benchmarks/bench_gelu_gemm.py > $O/bench.log 2>&1
rc=$?; tail -n 2 $O/bench.log; exit $rc
