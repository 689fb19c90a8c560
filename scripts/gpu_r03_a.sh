# Round 3, call A: the ADVICE-fix GPU tests, then prefill-GEMM diagnostics
# (WQ4_PF_DIAG builds timed in one process, tools/pf_variants.py).
set -o pipefail
mkdir -p gpurun_out/r03a
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_q4_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "large_range or n1312 or decode_step or out_of_decode or ffn_numerics" > gpurun_out/r03a/tests.log 2>&1 || { tail -30 gpurun_out/r03a/tests.log; exit 1; }
tail -3 gpurun_out/r03a/tests.log
L="whisper-burn_amd/lib/libwq4.so whisper-burn_amd/pfdiag/1/libwq4.so whisper-burn_amd/pfdiag/2/libwq4.so whisper-burn_amd/pfdiag/3/libwq4.so whisper-burn_amd/pfdiag/4/libwq4.so"
ROWS=48000 timeout -k 10 240 python -u tools/pf_variants.py $L > gpurun_out/r03a/pf48000.log 2>&1 || exit 1
ROWS=1500 ROUNDS=9 timeout -k 10 240 python -u tools/pf_variants.py $L > gpurun_out/r03a/pf1500.log 2>&1 || exit 1
cat gpurun_out/r03a/pf48000.log gpurun_out/r03a/pf1500.log
