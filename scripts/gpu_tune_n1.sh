#!/bin/bash
# Thorough TunableOp search for the N = 1 GEMM shapes (forward + TN dgrad, no LM head), merged
# into a copy of the table, then the default bench with the new and the old table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/tune_n1
mkdir -p $O
T=profiles/tunableop/gfx950_gpt345m_results.csv
cp $T $O/table_old.csv
SMDT_TUNE_N1_FORWARD=1 timeout -k 10 700 python -u scripts/tune_gemm_shapes.py --out $O/n1.csv --tune-ms 150 --iters 20 > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
python scripts/tune_gemm_shapes.py --out $O/n1.csv --merge-only > /dev/null && cp $T $O/table_new.csv
timeout -k 10 300 python -u bench.py > $O/bench_new.log 2>&1 || { tail -20 $O/bench_new.log; exit 1; }
cp $O/table_old.csv $T
timeout -k 10 300 python -u bench.py > $O/bench_old.log 2>&1 || { tail -20 $O/bench_old.log; exit 1; }
cp $O/table_new.csv $T
timeout -k 10 300 python -u bench.py > $O/bench_new2.log 2>&1 || { tail -20 $O/bench_new2.log; exit 1; }
for f in bench_new bench_old bench_new2; do tail -1 $O/$f.log | cut -c1-160; done
