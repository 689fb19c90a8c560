# xattn_main attribution at HEAD (V2 removed): isolated timings of the
# WA_XATTN_DIAG builds and the phase stamps of workgroup (0, 0); then the
# decode at 1 / 3 groups against the default 2 (32 clips).
set -o pipefail
O=gpurun_out/r05f; mkdir -p $O; export TMPDIR=/tmp
for b in whisper-burn_amd/build/xmicro/*; do
  echo "== $(basename $b)"
  WA_XATTN_SMALL_ROWS=0 timeout -k 10 60 ./$b 100 | grep -E '"rows": (16|32), ' || exit 1
done > $O/xattn_micro.log 2>&1; rc=$?; cat $O/xattn_micro.log; [ $rc -eq 0 ] || exit $rc
b() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/$n.json > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['phase_ms'])"
}
b base && b g1 WA_DECODE_GROUPS=1 && b g3 WA_DECODE_GROUPS=3
