# A/B in one box: the default EOT-polled decode loop vs --fixed-length (no per-step D2H poll)
mkdir -p gpurun_out
export TMPDIR=/tmp
for arm in "" "--fixed-length" "" "--fixed-length"; do
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline $arm > gpurun_out/eot_ab.log 2>&1 || exit $?
  grep '^{' gpurun_out/eot_ab.log | python -c "import json,sys; d=json.load(sys.stdin); p=d['phase_ms']; print('[$arm] RTF', d['value'], 'dec/step ms', round(p['decode_ms']/224,4))"
done
