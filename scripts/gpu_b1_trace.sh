# One clip (BASELINE config 3) under a kernel trace: per-kernel time of the
# graph-replayed one-row decode step.
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r02}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/b1_$R -o run --output-format csv -- python3 bench.py --clips-per-gpu 1 --steps 1 --warmup 1 --max-tokens 64 --fixed-length --no-cpu-baseline > gpurun_out/b1_$R.log 2>&1 || exit $?
f=$(ls gpurun_out/b1_$R/*/run_kernel_stats.csv gpurun_out/b1_$R/run_kernel_stats.csv 2>/dev/null | head -1)
python3 scripts/kstats.py $f 25 | tee gpurun_out/b1_kstats_$R.txt
rm -f $(ls gpurun_out/b1_$R/*/run_kernel_trace.csv gpurun_out/b1_$R/run_kernel_trace.csv 2>/dev/null)
