#!/bin/bash
# Round 4: two-rank rehearsals on ONE GPU over Gloo (RCCL refuses two ranks on one device) of
# the N = 8 building blocks with real kernels: pp2 under zbh2 and zbh1 (deferred / held W GEMMs,
# p2p), tp2 + SP (ring collective-matmul with the norms' gather slots).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
O=gpurun_out/r4aa
mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$R/$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 2 "$R/$O/$name.log" | cut -c1-700
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
RUN="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611"
export SMDT_BENCH_BACKEND=gloo
step pp2_zbh2 240 $RUN bench.py --gpus 2 --tp 1 --pp 2 --steps 3 --warmup 2 --tunableop 0 --seqs-per-gpu 16 --pp-schedule zbh2
step pp2_zbh1 240 $RUN bench.py --gpus 2 --tp 1 --pp 2 --steps 3 --warmup 2 --tunableop 0 --seqs-per-gpu 16 --pp-schedule zbh1
step tp2_sp 240 $RUN bench.py --gpus 2 --tp 2 --pp 1 --steps 3 --warmup 2 --tunableop 0 --seqs-per-gpu 16
echo DONE
