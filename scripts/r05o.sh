# prompt graphs: full GPU suite + smoke, then the pipelined bench (10 steps)
set -o pipefail
O=gpurun_out/r05o; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1; rc=$?
tail -4 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 --json-out $O/pipe.json > $O/pipe.log 2>&1 || { tail -5 $O/pipe.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/pipe.json')); print('pipe', d['value'], d['phase_ms'])"
