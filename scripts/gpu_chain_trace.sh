# The default bench workload (GROUPS_N: force the decode-group count) under a kernel trace: per-kernel time of the
# graph-replayed decode step (scripts/trace_gaps.py).
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r02}
${GROUPS_N:+env WA_DECODE_GROUPS=$GROUPS_N} timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/chain_$R -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --max-tokens 24 --fixed-length --no-cpu-baseline > gpurun_out/chain_$R.log 2>&1 || exit $?
f=$(ls gpurun_out/chain_$R/*/run_kernel_trace.csv gpurun_out/chain_$R/run_kernel_trace.csv 2>/dev/null | head -1)
python3 scripts/trace_gaps.py $f gpurun_out/chain_gaps_$R.json
python3 scripts/trace_by_grid.py $f "${GRID_RX:-skinny|q4_gemm_decode|xattn}" gpurun_out/chain_grid_$R.json
rm -f $f
