#!/bin/bash
# Round 4, second session: per-rank N = 8 / GPT-3 TP4 emulation + schedule prediction, and the
# N = 4 rehearsal-stall isolation (Gloo CUDA-tensor reduce-scatter probe, traced rehearsal).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4b
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 12 "$R/$O/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step predict 900 python -u benchmarks/predict_scaling.py --out $O/predict
# Gloo, CUDA tensors, N processes on the one GPU: 75 async reduce-scatters of 16 MB in the same
# order on every rank (exit 3 = the probe's own stall watchdog fired; the step continues)
for n in 2 4; do
  echo "=== gloo_probe_n$n"
  timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29600 + n)) benchmarks/gloo_cuda_probe.py --buckets 75 --mb 16 --limit 90 > $O/gloo_probe_n$n.log 2>&1
  echo "rc=$?"; grep '^{' $O/gloo_probe_n$n.log || tail -5 $O/gloo_probe_n$n.log
done
# the round-3 rehearsal again, with every rank's collective issue order traced
echo "=== rehearse_n4"
SMDT_BENCH_BACKEND=gloo SMDT_COLLECTIVE_LOG=$R/$O/clog SMDT_BENCH_DUMP_AFTER=100 timeout -k 10 160 \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29611 \
  bench.py --gpus 4 --steps 2 --warmup 1 --tunableop 0 --seqs-per-gpu 8 > $O/rehearse_n4.log 2>&1
echo "rc=$?"; grep '^{' $O/rehearse_n4.log | cut -c1-300; wc -l $O/clog.rank* 2>/dev/null
echo DONE
