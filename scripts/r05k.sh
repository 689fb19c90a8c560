# pipelined bench with one decode group vs two (10 steps)
set -o pipefail
O=gpurun_out/r05k; mkdir -p $O; export TMPDIR=/tmp
b() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 --json-out $O/$n.json "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); p=d.get('pipeline') or {}; print('$n', d['value'], d['phase_ms'], p.get('overlap_layers'), p.get('masked_ms'))"
}
WA_DECODE_GROUPS=1 b g1p && b g2p && WA_DECODE_GROUPS=1 WA_ENC_CUS=64 b g1p64 && WA_DECODE_GROUPS=3 b g3p
