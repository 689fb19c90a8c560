# xattn_out merge rewrite + xattn_main V2 loop: parity (xattn tests incl. the
# V2 bit-identity), isolated timings, then bench A/B at 32 clips:
# base / WA_XATTN_MAIN=1 / 12 splits / 12 splits + V2.
set -o pipefail
O=gpurun_out/r05e; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_xattn_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for b in whisper-burn_amd/build/xmicro/*; do
  echo "== $(basename $b)"
  WA_XATTN_SMALL_ROWS=0 timeout -k 10 60 $b 100 | grep -E "main_us|main_v2" || exit 1
done 2>&1 | tee $O/xattn_micro.log
b() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/$n.json > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['phase_ms'])"
}
b base && b v2 WA_XATTN_MAIN=1 && b s12 WQ4_LIB_DIR=$PWD/whisper-burn_amd/diag/s12 && \
  b s12v2 WQ4_LIB_DIR=$PWD/whisper-burn_amd/diag/s12 WA_XATTN_MAIN=1 && b base2
