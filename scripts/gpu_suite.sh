# Full GPU parity suite (verbose, with the tests' own prints), then smoke().
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu -s --timeout 300 --timeout-method thread -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|worst|tokens equal|FAILED" gpurun_out/pytest_gpu.log | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
exit $rc
