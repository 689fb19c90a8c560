# One call: GPU parity tests, smoke(), then the default bench line.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
cat gpurun_out/smoke.log
timeout -k 10 600 python bench.py --json-out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
