# encoder kernel stats at full width (sequential transcribe, 8 tokens: the
# encoder dominates), 4 encoder runs
set -o pipefail
O=gpurun_out/r05z; mkdir -p $O; export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/stats -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --sequential --max-tokens 8 > $GRAFT_REPO_ROOT/$O/stats.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python3 scripts/kstats.py $(ls $O/stats/*/run_kernel_stats.csv $O/stats/run_kernel_stats.csv 2>/dev/null | head -1) 16
