# xattn_main scores from the fetched registers (WA_XATTN_SREG=1 variant):
# isolated timing, the xattn parity tests on the variant library, bench A/B.
set -o pipefail
O=gpurun_out/r05l; mkdir -p $O; export TMPDIR=/tmp
for b in diag0 v_sreg; do
  echo "== $b"; WA_XATTN_SMALL_ROWS=0 timeout -k 10 60 ./whisper-burn_amd/build/xmicro/$b 100 | grep '"small"' || exit 1
done 2>&1 | tee $O/xattn_micro.log
WQ4_LIB_DIR=$PWD/whisper-burn_amd/diag/sreg timeout -k 10 400 python -u -m pytest tests/test_xattn_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
b() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 --sequential --json-out $O/$n.json "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['phase_ms'])"
}
b base && WQ4_LIB_DIR=$PWD/whisper-burn_amd/diag/sreg b sreg && b base2
