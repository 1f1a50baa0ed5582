#!/bin/bash
# One parameterised GPU session on a single MI355X (run from the repo root on the gpurun box):
#
#   OUT=gpurun_out/<name> STEPS="tests smoke bench bench prof" bash scripts/gpu_session.sh
#
# STEPS is a space-separated list of the named steps below, run in order. Every GPU step runs
# under its own `timeout -k 10`, writes `$OUT/<step>[_<i>].log`, and the session stops at the
# first step that fails (a fault, abort or time limit ends the call: nothing more touches the GPU).
#
# Knobs: TESTS (pytest paths, default `tests`), BENCH_ARGS (extra bench.py flags),
# BSTEPS / BWARM (bench steps / warmup, default 20 / 5), PROF_ARGS (bench flags for the profile),
# PMC (counter list for the `pmc` step), CMD (free command for the `cmd` step).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=${OUT:-gpurun_out/session}
mkdir -p "$O"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
declare -A SEEN
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  local n=${SEEN[$name]:-0}; SEEN[$name]=$((n + 1))
  [ "$n" -gt 0 ] && name="${name}_$n"
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 3 "$R/$O/$name.log" | cut -c1-600
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
}
BS=${BSTEPS:-20}; BW=${BWARM:-5}
for s in ${STEPS:-tests smoke bench}; do
  case $s in
    tests) run pytest_gpu 900 python -u -m pytest -q -x --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests} ;;
    smoke) run smoke 180 python __graft_entry__.py smoke ;;
    bench) run bench 400 python bench.py --steps $BS --warmup $BW ${BENCH_ARGS:-} ;;
    attn) run attn 150 python benchmarks/bench_attention.py --b 64 --sdpa 0 --dropout 0.1 ;;
    vision) run vision_r50 500 python benchmarks/bench_vision.py --model resnet50 --size 224 --batch 64 --steps 20 --warmup 5
            run vision_swin 500 python benchmarks/bench_vision.py --model swin_b --size 128 --batch 40 --steps 20 --warmup 5 ;;
    prof)
      cd /tmp
      run prof 400 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv -- \
        python3 "$R/bench.py" --steps 3 --warmup 3 ${PROF_ARGS:-${BENCH_ARGS:-}}
      cd "$R"
      f=$(find "$O/prof" -name '*kernel_trace.csv' | head -n 1)
      python scripts/ktrace_steps.py "$f" 40 > "$O/last_step_breakdown.txt" && head -n 20 "$O/last_step_breakdown.txt"
      find "$O/prof" -name '*kernel_trace.csv' -delete ;;
    pmc)
      cd /tmp
      run pmc 120 rocprofv3 --pmc ${PMC} --kernel-trace --stats -d "$R/$O/pmc" -o run --output-format csv -- ${CMD}
      cd "$R" ;;
    cmd) run cmd ${CMD_TIMEOUT:-300} bash -c "${CMD}" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo DONE
