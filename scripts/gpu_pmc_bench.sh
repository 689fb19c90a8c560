# FETCH_SIZE / WRITE_SIZE passes (short run, split by grid), then the bench
# line reading that summary (profiles/pmc_traffic.json is copied back by hand).
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r01}
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-include-regex "q4_gemm|xattn" -d gpurun_out/pmc_${C}_$R -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --max-tokens 8 --no-cpu-baseline > gpurun_out/pmc_${C}_$R.log 2>&1 || exit $?
  echo "pmc $C done"
done
python3 scripts/pmc_summary.py $R gpurun_out/pmc_traffic_$R.json > gpurun_out/pmc_summary_$R.log || exit 1
head -c 300 gpurun_out/pmc_FETCH_SIZE_$R/*/run_counter_collection.csv 2>/dev/null | head -2 || true
rm -f gpurun_out/pmc_*_$R/*/run_counter_collection.csv gpurun_out/pmc_*_$R/run_counter_collection.csv
cp gpurun_out/pmc_traffic_$R.json profiles/pmc_traffic.json
timeout -k 10 600 python bench.py --json-out gpurun_out/bench_$R.json > gpurun_out/bench_$R.log 2>&1 || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_$R.json')); print(d['value'], d['roofline'])"
