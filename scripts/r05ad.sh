# pipelined transcribe: the masked part's fill of the decode (k adapts to
# fill x the last decode / the masked time per layer), 10 steps each
set -o pipefail
O=gpurun_out/r05ad${SUF}; mkdir -p $O; export TMPDIR=/tmp
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 --json-out $O/$n.json > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); p=d['phase_ms']; print('$n', d['value'], p, d['pipeline']['overlap_layers'], round(d['pipeline']['masked_ms'],1))"
}
run f098 WA_ENC_FILL=0.98 && run f100 WA_ENC_FILL=1.0 && run f102 WA_ENC_FILL=1.02 && run f092 A=1 && run f100b WA_ENC_FILL=1.0
