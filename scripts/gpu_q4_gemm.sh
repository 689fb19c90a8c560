# Q4 operator GPU tests, then the encoder GEMM probe with counters.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_q4_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/q4_tests.log 2>&1; rc=$?
tail -3 gpurun_out/q4_tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_gemm_prof.sh
