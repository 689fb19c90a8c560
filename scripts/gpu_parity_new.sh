# Round-2 parity additions: direct kernel tests and full-size fixture tests.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_full_size_gpu.py -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/parity_new.log 2>&1; rc=$?
tail -40 gpurun_out/parity_new.log
exit $rc
