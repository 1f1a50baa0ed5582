#!/bin/bash
# North-star and like-for-like configs on one MI355X with the current bench.py (self-labelled JSON).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/ns
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/ns/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 2 "gpurun_out/ns/$name.log"
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step gpt3_6p7b_1gpu 480 python bench.py --num-layers 32 --hidden-size 4096 --num-attention-heads 32 --seq-length 2048 --seqs-per-gpu 4 --micro-batch-size 4 --steps 5 --warmup 2
step gpt2_small_1gpu 300 python bench.py --num-layers 12 --hidden-size 768 --num-attention-heads 12 --seqs-per-gpu 48 --micro-batch-size 12 --grad-accum 4 --steps 10 --warmup 3
LLAMA=1 STEPS=20 LSTEPS=8 bash scripts/gpu_alpaca.sh > gpurun_out/ns/alpaca.log 2>&1; rc=$?; tail -n 8 gpurun_out/ns/alpaca.log; cp -r gpurun_out/alpaca gpurun_out/ns/ 2>/dev/null; echo "alpaca rc=$rc"
echo DONE
