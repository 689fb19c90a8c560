# Kernel trace of a one-group decode (32 clips, 16 tokens): busy time vs gaps in the launch chain.
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r01}
WA_DECODE_GROUPS=${GROUPS_N:-1} timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/chain_$R -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --max-tokens 16 --fixed-length --no-cpu-baseline > gpurun_out/chain_$R.log 2>&1 || exit $?
f=$(find gpurun_out/chain_$R -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_gaps.py "$f" gpurun_out/chain_gaps_$R.json
rm -f "$f"
