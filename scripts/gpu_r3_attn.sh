#!/bin/bash
# Attention microbenchmark at the bench's shape (B64 S1024 H16 D64 causal, dropout 0.1 and 0)
# and the LLaMA-7B shape (D128), ours vs torch SDPA.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r3_attn
mkdir -p $O
timeout -k 10 200 python -u benchmarks/bench_attention.py --b 64 --h 16 --s 1024 --d 64 --dropout 0.1 --sdpa 0 > $O/gpt345m_drop.log 2>&1 || { tail -20 $O/gpt345m_drop.log; exit 1; }
timeout -k 10 200 python -u benchmarks/bench_attention.py --b 64 --h 16 --s 1024 --d 64 > $O/gpt345m_nodrop.log 2>&1 || { tail -20 $O/gpt345m_nodrop.log; exit 1; }
timeout -k 10 200 python -u benchmarks/bench_attention.py --b 4 --h 32 --s 2048 --d 128 > $O/llama_d128.log 2>&1 || { tail -20 $O/llama_d128.log; exit 1; }
tail -n 3 $O/*.log
