# Bench RTF under a list of environment settings (ENVLIST, ';'-separated
# assignments per run), e.g. ENVLIST="WA_DECODE_GROUPS=2;WA_DECODE_GROUPS=3".
IFS=';' read -ra RUNS <<< "$ENVLIST"
i=0
for R in "${RUNS[@]}"; do
  i=$((i+1))
  env $R timeout -k 10 400 python bench.py --no-cpu-baseline --json-out gpurun_out/bench_e$i.json > gpurun_out/bench_e$i.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_e$i.json')); print('$R', 'RTF', d['value'], d['phase_ms'])"
done
