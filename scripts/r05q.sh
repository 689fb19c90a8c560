# phase offset between the two decode groups (sequential decode, 5 steps each)
set -o pipefail
O=gpurun_out/r05q; mkdir -p $O; export TMPDIR=/tmp
b() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 --sequential --json-out $O/$n.json "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['phase_ms'])"
}
b s0 && WA_GROUP_SKEW_US=25 b s25 && WA_GROUP_SKEW_US=50 b s50 && WA_GROUP_SKEW_US=100 b s100 && WA_GROUP_SKEW_US=1700 b s1700 && b s0b
