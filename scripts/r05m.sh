# second head tile's qt with a zero row (one address + immediates): isolated
# xattn timing, xattn + model parity, sequential and pipelined bench.
set -o pipefail
O=gpurun_out/r05m; mkdir -p $O; export TMPDIR=/tmp
WA_XATTN_SMALL_ROWS=0 timeout -k 10 60 ./whisper-burn_amd/build/xmicro/diag0 100 | grep '"small"' | tee $O/xattn_micro.log || exit 1
timeout -k 10 400 python -u -m pytest tests/test_xattn_gpu.py tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
b() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 --json-out $O/$n.json "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['phase_ms'])"
}
b seq --sequential && b pipe
