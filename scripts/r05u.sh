# masked encoder GEMMs at one workgroup per CU (LDS pad), 32 / 64 masked CUs
set -o pipefail
O=gpurun_out/r05u; mkdir -p $O; export TMPDIR=/tmp
b() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 --json-out $O/$n.json "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); p=d.get('pipeline') or {}; print('$n', d['value'], d['phase_ms'], p.get('overlap_layers'), p.get('masked_ms'))"
}
b base && WA_ENC_LDS_PAD=20000 b pad32 && WA_ENC_LDS_PAD=20000 WA_ENC_CUS=64 b pad64 && WA_ENC_LDS_PAD=20000 WA_ENC_CUS=48 b pad48
