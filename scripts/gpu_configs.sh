# BASELINE.json configs 2, 3 and 5 beside the config-4 shard bench line (one bench run each)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r01}
run() {  # name, bench args
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --json-out gpurun_out/cfg_${n}_$R.json "$@" > gpurun_out/cfg_${n}_$R.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/cfg_${n}_$R.json')); print('$n', d['value'], d['unit'], d['phase_ms'])"
}
run c2_medium_b1 --variant medium --clips-per-gpu 1
run c3_large_v3_b1 --clips-per-gpu 1
run c5_large_v3_f16w --weights f16
run c5_large_v3_f16w_b1 --weights f16 --clips-per-gpu 1
run c4_precision_f16 --precision f16
