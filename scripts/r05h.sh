# Pipelined transcribes: parity, then the bench pipelined (default) against
# --sequential, then the masked-encoder probe at 40 / 48 CUs and with
# high-priority decode streams.
set -o pipefail
O=gpurun_out/r05h; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_pipeline_gpu.py "tests/test_full_size_gpu.py::test_full_size_tokens_pipelined" -x -v -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
b() {  # name, env / args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/$n.json "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['phase_ms'], d.get('pipeline'))"
}
b pipe && b seq --sequential && WA_ENC_CUS=48 b pipe48 && WA_ENC_CUS=40 b pipe40 && WA_GROUP_PRIO=1 WA_ENC_CUS=64 b pipe64prio
