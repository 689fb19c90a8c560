# masked encoder CUs 24 / 40 / 48 against 32 at fill 0.98 (final tree), 10 steps
set -o pipefail
O=gpurun_out/r05ae; mkdir -p $O; export TMPDIR=/tmp
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 --json-out $O/$n.json > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); p=d['phase_ms']; print('$n', d['value'], p, d['pipeline']['overlap_layers'], round(d['pipeline']['masked_ms'],1))"
}
run c32 A=1 && run c40 WA_ENC_CUS=40 && run c48 WA_ENC_CUS=48 && run c24 WA_ENC_CUS=24 && run c32b A=1
