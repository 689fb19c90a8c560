# A/B of the decode GEMM plans (8-wave whole-K vs 4-wave split-K): tests, microbench, model profile
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
for w8 in ${W8S:-1 0}; do
  echo "== WQ4_DECODE_W8=$w8"
  WQ4_DECODE_W8=$w8 timeout -k 10 300 python whisper-burn_amd/tools/q4_bench.py --decode-only --iters 50 > gpurun_out/q4_dec_w8_$w8.log 2>&1 || exit $?
  grep f16x2 gpurun_out/q4_dec_w8_$w8.log
  WQ4_DECODE_W8=$w8 timeout -k 10 600 python bench.py --steps 1 --warmup 1 --max-tokens 64 --no-cpu-baseline > gpurun_out/bench_w8_$w8.log 2>&1 || exit $?
  grep '^{' gpurun_out/bench_w8_$w8.log | python -c "import json,sys; d=json.load(sys.stdin); print('RTF', d['value'], d['phase_ms'], d['roofline_decode_gemm']['avg_us'])"
done
