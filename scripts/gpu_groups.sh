# decode groups A/B: GPU tests, then a 64-token bench per WA_DECODE_GROUPS
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
for G in ${GROUPS_LIST:-1 2 4}; do
  WA_DECODE_GROUPS=$G timeout -k 10 600 python bench.py --steps 1 --warmup 1 --max-tokens ${TOKENS:-64} --no-cpu-baseline > gpurun_out/bench_g$G.log 2>&1 || exit $?
  grep '^{' gpurun_out/bench_g$G.log | python -c "import json,sys; d=json.load(sys.stdin); print('G=$G RTF', d['value'], d['phase_ms'])"
done
