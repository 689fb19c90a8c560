# rocprofv3 kernel trace of a short bench run, cross-attention kernels split by
# grid: the probe-shape launches (all clips in one launch) are the ones the
# bench's roofline avg_us times with HIP events.
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r01}
timeout -k 10 600 rocprofv3 --kernel-trace --kernel-include-regex "xattn" -d gpurun_out/xtrace_$R -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --max-tokens ${TOKENS:-16} --no-cpu-baseline --json-out gpurun_out/xtrace_bench_$R.json > gpurun_out/xtrace_$R.log 2>&1 || exit $?
f=$(find gpurun_out/xtrace_$R -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_by_grid.py "$f" xattn gpurun_out/xattn_by_grid_$R.json
python3 -c "import json; d=json.load(open('gpurun_out/xtrace_bench_$R.json')); print('bench probe avg_us (xattn_q+main+out, HIP events):', d['roofline_cross_attention']['avg_us'])"
rm -f "$f"
