# GPU tests, then 64-token fixed-length decode sweeps over env knobs (one config per line of $CFGS: "G S EXTRA_ENV")
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
i=0
while read -r G S EXTRA; do
  [ -z "$G" ] && continue
  i=$((i+1))
  env WA_DECODE_GROUPS=$G WA_XATTN_SPLITS=$S $EXTRA timeout -k 10 300 python bench.py --steps 1 --warmup 1 --max-tokens 64 --fixed-length --no-cpu-baseline > gpurun_out/sw_$i.log 2>&1 || exit $?
  grep '^{' gpurun_out/sw_$i.log | python -c "import json,sys; d=json.load(sys.stdin); p=d['phase_ms']; print('G=$G S=$S $EXTRA RTF', d['value'], 'dec/step ms', round(p['decode_ms']/64,3), 'enc', p['encoder_ms'])"
done <<< "$CFGS"
