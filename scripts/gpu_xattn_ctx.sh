# cross-attention in model context: short bench per decode-group count, then a kernel trace at G=1
mkdir -p gpurun_out
export TMPDIR=/tmp
for G in ${GROUPS_LIST:-1 2}; do
  WA_DECODE_GROUPS=$G timeout -k 10 600 python bench.py --steps 2 --warmup 1 --max-tokens ${TOKENS:-32} --fixed-length --no-cpu-baseline > gpurun_out/bench_g$G.log 2>&1 || exit $?
  grep '^{' gpurun_out/bench_g$G.log | python -c "import json,sys; d=json.load(sys.stdin); print('G=$G RTF', d['value'], d['phase_ms'], 'xattn us', d['roofline_cross_attention']['avg_us'])"
done
WA_DECODE_GROUPS=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g1 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --max-tokens 16 --fixed-length --no-cpu-baseline > gpurun_out/prof_g1.log 2>&1 || exit $?
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/prof_g1/run_kernel_stats.csv')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:16]:
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.2f}us {float(r['TotalDurationNs'])/1e6:8.2f}ms")
PY
