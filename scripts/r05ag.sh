# decoder self-attention with 8 waves per (head, clip) at Tq = 1: parity
# (kernels, model, full size, pipeline), then sequential and pipelined bench
set -o pipefail
O=gpurun_out/r05ag; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_full_size_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
b() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 --json-out $O/$n.json "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['phase_ms'])"
}
b seq --sequential && b pipe && b pipe2
