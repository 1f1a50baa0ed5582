set -u
O=gpurun_out/r5_miopen_check; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2; do
  t0=$(date +%s)
  timeout -k 10 600 python benchmarks/bench_vision.py --model resnet50 --size 224 --batch 64 --steps 20 --warmup 5 > $O/r50_default_$i.log 2>&1 || exit $?
  echo "r50 default run $i wall $(( $(date +%s) - t0 ))s: $(grep -h '"metric"' $O/r50_default_$i.log | cut -c1-150)"
done
echo "MIOPEN_USER_DB_PATH dir: $(ls ~/.cache/smdt_amd/miopen 2>&1)"
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_bench_vision.py tests/test_vision_models.py > $O/tests.log 2>&1; echo "tests rc=$?"; tail -2 $O/tests.log
