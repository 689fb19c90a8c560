# logits kernel with the table two chunks ahead: parity (kernel, model,
# full-size) and the trace-free in-model duration, then the pipelined bench
set -o pipefail
O=gpurun_out/r05v; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_full_size_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
b() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 --json-out $O/$n.json "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['phase_ms'])"
}
b seq --sequential && b pipe
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/stats -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline --sequential --max-tokens 32 > $GRAFT_REPO_ROOT/$O/stats.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python3 scripts/kstats.py $(ls $O/stats/*/run_kernel_stats.csv $O/stats/run_kernel_stats.csv 2>/dev/null | head -1) 8
