# round 6: the Megatron model-form flags, the Switch MLP and --use-cpu-initialization on the GPU,
# then the full GPU suite and smoke on the same tree
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/${OUT:-r6_flags}; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 1 $O/$n.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
run variants 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_model_gpu.py -k "model_form_variants or switch_mlp or cpu_initialization"
run pytest_gpu 900 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests
run smoke 180 python __graft_entry__.py smoke
echo DONE
