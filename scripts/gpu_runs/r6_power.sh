# round 6: power and clocks while the N = 1 bench step runs (is the full-chip step power-capped?)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
O=$R/gpurun_out/r6_power; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 5 20 rocm-smi --showpower --showclocks --showmaxpower > $O/idle.txt 2>&1 || true
( for i in $(seq 1 60); do echo "--- $(date +%T.%N)"; timeout -k 2 5 rocm-smi --showpower --showclocks 2>&1 | grep -iE "power|sclk|mclk|fclk" ; sleep 0.5; done ) > $O/during.txt 2>&1 &
MON=$!
timeout -k 10 300 python bench.py --steps 60 --warmup 5 > $O/bench.log 2>&1
rc=$?
kill $MON 2>/dev/null; wait $MON 2>/dev/null
tail -n 1 $O/bench.log | cut -c1-160
grep -iE "power|sclk" $O/during.txt | sort | uniq -c | sort -rn | head -20
exit $rc
