# Round-end measurement set: full bench line, rocprofv3 kernel-trace summary of
# the same command, then separate FETCH_SIZE / WRITE_SIZE PMC passes (short run).
# Big per-dispatch CSVs are reduced on the box (gpurun_out/ must stay < 64 MiB).
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r01}
timeout -k 10 900 python bench.py --json-out gpurun_out/bench_$R.json > gpurun_out/bench_$R.log 2>&1 || exit $?
tail -1 gpurun_out/bench_$R.log
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$R -o run --output-format csv -- python3 bench.py --no-cpu-baseline --json-out gpurun_out/bench_prof_$R.json > gpurun_out/prof_$R.log 2>&1 || exit $?
rm -f gpurun_out/prof_$R/run_kernel_trace.csv
echo "kernel-trace pass done"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 900 rocprofv3 --pmc $C --kernel-include-regex "q4_gemm|xattn" -d gpurun_out/pmc_${C}_$R -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --max-tokens 8 --no-cpu-baseline > gpurun_out/pmc_${C}_$R.log 2>&1 || exit $?
  echo "pmc $C done"
done
python3 scripts/pmc_summary.py $R gpurun_out/pmc_traffic_$R.json > gpurun_out/pmc_summary_$R.log && rm -f gpurun_out/pmc_*_$R/run_counter_collection.csv
du -sh gpurun_out
