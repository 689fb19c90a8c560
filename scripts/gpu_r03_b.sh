# Round 3, call B: the encoder GEMM ring kernel -- bit identity vs the
# prefill tile kernel, the Q4 operator tests, then timing (old vs new, one
# process) and a kernel trace.
set -o pipefail
mkdir -p gpurun_out/r03b
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_q4_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "enc_kernel or whisper_shapes or large_range or n1312 or decode_step or out_of_decode" > gpurun_out/r03b/tests.log 2>&1 || { tail -40 gpurun_out/r03b/tests.log; exit 1; }
tail -3 gpurun_out/r03b/tests.log
ROWS=48000 timeout -k 10 240 python -u tools/enc_ab.py > gpurun_out/r03b/ab48000.log 2>&1 || { cat gpurun_out/r03b/ab48000.log; exit 1; }
ROWS=1500 ROUNDS=9 timeout -k 10 240 python -u tools/enc_ab.py > gpurun_out/r03b/ab1500.log 2>&1 || exit 1
cat gpurun_out/r03b/ab48000.log gpurun_out/r03b/ab1500.log
