# Pipelined bench at the driver's step counts: masked-stream CU count and a
# decode confined to the other CUs.
set -o pipefail
O=gpurun_out/r05i; mkdir -p $O; export TMPDIR=/tmp
b() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 --json-out $O/$n.json "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); p=d.get('pipeline') or {}; print('$n', d['value'], d['phase_ms'], p.get('overlap_layers'), p.get('masked_ms'))"
}
b p32 && WA_DECODE_CUMASK=32 b p32x && WA_ENC_CUS=24 b p24 && WA_ENC_CUS=48 WA_DECODE_CUMASK=48 b p48x && WA_ENC_CUS=64 WA_DECODE_CUMASK=64 b p64x
