# Round-end evidence for profiles/ (ROUND, default r02): GPU parity suite,
# smoke(), the in-graph decode trace (2 decode groups, as the bench runs),
# PMC FETCH_SIZE / WRITE_SIZE passes, kernel-trace stats of the bench, the
# encoder Q4 GEMM MFMA counters, then the final bench line reading the PMC
# and in-graph summaries.  Everything lands in gpurun_out/$ROUND.
R=${ROUND:-r02}
O=gpurun_out/$R
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu -s --timeout 300 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed" $O/pytest_gpu.log | tail -2
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
ROUND=$R bash scripts/gpu_chain_trace.sh > $O/chain.txt 2>&1 || exit $?
cp gpurun_out/chain_gaps_$R.json gpurun_out/chain_grid_$R.json $O/
python3 scripts/in_graph_summary.py gpurun_out/chain_grid_$R.json large_v3 q4_0 f16x2 32 $O/xattn_in_graph.json || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-include-regex "q4_gemm|xattn" -d gpurun_out/pmc_${C}_$R -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --max-tokens 8 --no-cpu-baseline > gpurun_out/pmc_${C}_$R.log 2>&1 || exit $?
  echo "pmc $C done"
done
python3 scripts/pmc_summary.py $R $O/pmc_traffic.json > $O/pmc_summary.log || exit 1
rm -f gpurun_out/pmc_*_$R/*/run_counter_collection.csv gpurun_out/pmc_*_$R/run_counter_collection.csv
cp $O/pmc_traffic.json profiles/pmc_traffic.json
cp $O/xattn_in_graph.json profiles/xattn_in_graph.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/stats_$R -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --json-out $O/bench_under_rocprof.json > $O/stats.log 2>&1 || exit $?
f=$(ls gpurun_out/stats_$R/*/run_kernel_stats.csv gpurun_out/stats_$R/run_kernel_stats.csv 2>/dev/null | head -1)
cp $f $O/kernel_stats.csv
rm -f gpurun_out/stats_$R/*/run_kernel_trace.csv gpurun_out/stats_$R/run_kernel_trace.csv
ROUND=$R POLICY=0 bash scripts/gpu_gemm_prof.sh > $O/q4_gemm_mfma.txt 2>&1 || exit $?
rm -f gpurun_out/gemm_*/*/run_kernel_trace.csv gpurun_out/gemm_pmc*/*/run_counter_collection.csv gpurun_out/gemm_*/run_kernel_trace.csv gpurun_out/gemm_pmc*/run_counter_collection.csv
timeout -k 10 600 python bench.py --json-out $O/bench.json > $O/bench.log 2>&1 || exit $?
tail -c 600 $O/bench.json
