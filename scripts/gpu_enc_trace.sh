# kernel trace of one encoder pass (32 clips), per-kernel summary
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/enc_trace -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --max-tokens 2 --fixed-length --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/enc_trace.log 2>&1 || exit $?
rm -f gpurun_out/enc_trace/run_kernel_trace.csv
python3 scripts/kstats.py gpurun_out/enc_trace/run_kernel_stats.csv 12
