mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
cat gpurun_out/smoke.log
timeout -k 10 300 python whisper-burn_amd/tools/q4_bench.py --quick --json gpurun_out/q4_bench.json > gpurun_out/q4_bench.log 2>&1 || exit $?
cat gpurun_out/q4_bench.log
