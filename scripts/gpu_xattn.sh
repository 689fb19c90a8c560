# cross-attention rework: focused parity tests first, then the full GPU suite, then a short bench
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_xattn_gpu.py -q -x > gpurun_out/pytest_xattn.log 2>&1; rc=$?
echo "pytest xattn rc=$rc"; tail -15 gpurun_out/pytest_xattn.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest gpu rc=$rc"; tail -8 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --max-tokens ${TOKENS:-32} --fixed-length --no-cpu-baseline \
  --json-out gpurun_out/bench_xattn.json > gpurun_out/bench_xattn.log 2>&1 || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/bench_xattn.json'))
print('RTF', d['value'], 'ms/step', d['ms_per_step'], d['phase_ms'])
print('xattn', d['roofline_cross_attention'])
print('dec', d['roofline_decode_gemm'])"
