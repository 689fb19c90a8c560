# Do CU-masked decode-group streams dispatch slowly?  Sequential decode with
# the groups' streams masked to CUs 1..255 / 32..255 / 128..255 (no encoder beside).
set -o pipefail
O=gpurun_out/r05n; mkdir -p $O; export TMPDIR=/tmp
b() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --sequential --json-out $O/$n.json "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['phase_ms'])"
}
b base && WA_DECODE_CUMASK=1 b m1 && WA_DECODE_CUMASK=32 b m32 && WA_DECODE_CUMASK=128 b m128
