ST="--num-layers 11 --emulate-last-stage --emulate-tp 2 --micro-batch-size 32 --grad-accum 8"
O=gpurun_out/r5_spmlp
timeout -k 10 300 python bench.py --steps 6 --warmup 2 $ST > $O/st_fused_1.log 2>&1 && \
SMDT_FUSED_BIAS_GELU=0 timeout -k 10 300 python bench.py --steps 6 --warmup 2 $ST > $O/st_unfused_1.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 6 --warmup 2 $ST > $O/st_fused_2.log 2>&1 && \
SMDT_FUSED_BIAS_GELU=0 timeout -k 10 300 python bench.py --steps 6 --warmup 2 $ST > $O/st_unfused_2.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 $ST --comm-stats 0 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 && cd $GRAFT_REPO_ROOT && \
f=$(find $O/prof -name '*kernel_trace.csv' | head -n 1) && python scripts/ktrace_steps.py "$f" 45 > $O/fused_last_step.txt 2>&1; find $O/prof -name '*kernel_trace.csv' -delete; grep -h '"metric"' $O/st_*.log | cut -c1-200
