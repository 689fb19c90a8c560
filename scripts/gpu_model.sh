# GPU session: Q4 tests, model parity tests, smoke, then a short bench.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python bench.py --clips-per-gpu 4 --steps 1 --warmup 1 --max-tokens 32 --cpu-rows 64 > gpurun_out/bench_small.log 2>&1 || exit $?
tail -3 gpurun_out/bench_small.log
