# Round-5 final set at HEAD: GPU suite + smoke, bench at the driver's counts
# (pipelined and --sequential), rocprofv3 kernel stats of one pipelined step.
set -o pipefail
O=gpurun_out/r05t; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1; rc=$?
tail -4 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --json-out $O/bench20.json > $O/bench20.log 2>&1 || { tail -5 $O/bench20.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench20.json')); print('pipe20', d['value'], d['phase_ms'], d['roofline']['frac'])"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --sequential --no-cpu-baseline --json-out $O/seq20.json > $O/seq20.log 2>&1 || { tail -5 $O/seq20.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/seq20.json')); print('seq20', d['value'], d['phase_ms'])"
OUT=r05t ROUND=r05 bash scripts/gpu.sh stats
