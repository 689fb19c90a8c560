# Bench RTF at 1..4 decode groups (WA_DECODE_GROUPS) for the default workload.
for G in ${GLIST:-1 2 3 4}; do
  WA_DECODE_GROUPS=$G timeout -k 10 400 python bench.py --no-cpu-baseline --json-out gpurun_out/bench_g$G.json > gpurun_out/bench_g$G.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_g$G.json')); print('groups $G RTF', d['value'], d['phase_ms'])"
done
