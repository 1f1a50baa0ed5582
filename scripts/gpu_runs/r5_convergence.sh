# GPT-2 345M loss curves on learnable synthetic data: the HIP-kernel path vs PyTorch reference
# ops on the same GPU (benchmarks/convergence.py), then the comparison table.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/${OUT:-r5_convergence}; mkdir -p $O
A="--steps ${STEPS:-400} ${CONV_ARGS:-}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "=== $n rc=$rc"; tail -n 2 $O/$n.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
run kernels 600 python -u benchmarks/convergence.py --kernels 1 $A --out $O/k1.json
SMDT_DISABLE_KERNELS=1 run reference 900 python -u benchmarks/convergence.py --kernels 0 $A --out $O/k0.json
# control: the kernel path with hipBLASLt for the MLP GEMMs and torch weight gradients (other
# summation orders, same math): its distance to the kernel run is the trajectory's own noise floor
SMDT_GEMM_TN=0 SMDT_FUSED_WGRAD=0 run control 600 python -u benchmarks/convergence.py --kernels 1 $A --out $O/k1b.json
python benchmarks/convergence.py --compare $O/k1.json $O/k0.json | tee $O/compare.md
python benchmarks/convergence.py --compare $O/k1.json $O/k1b.json --label "control: kernels, torch wgrad" | tee $O/compare_control.md
echo DONE
