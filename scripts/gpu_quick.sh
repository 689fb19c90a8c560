# quick loop: model/xattn GPU tests, then a 64-token fixed-length bench at G=1 and G=2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread ${TESTS:-} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
for G in ${GROUPS_LIST:-1 2}; do
  WA_DECODE_GROUPS=$G timeout -k 10 300 python bench.py --steps 1 --warmup 1 --max-tokens 64 --fixed-length --no-cpu-baseline > gpurun_out/quick_g$G.log 2>&1 || exit $?
  grep '^{' gpurun_out/quick_g$G.log | python -c "import json,sys; d=json.load(sys.stdin); p=d['phase_ms']; print('G=$G RTF', d['value'], 'dec/step ms', round(p['decode_ms']/64,3), p)"
done
