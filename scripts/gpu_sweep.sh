# Decode-path knob sweep: groups x xattn splits, fixed-length 64-token runs (phase_ms per config)
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in ${CFGS:-"1 8" "2 8" "1 4" "2 4"}; do
  set -- $cfg
  WA_DECODE_GROUPS=$1 WA_XATTN_SPLITS=$2 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --max-tokens ${TOKENS:-64} --fixed-length --no-cpu-baseline > gpurun_out/sweep_$1_$2.log 2>&1 || exit $?
  grep '^{' gpurun_out/sweep_$1_$2.log | python -c "import json,sys; d=json.load(sys.stdin); p=d['phase_ms']; print('G=$1 S=$2 RTF', d['value'], 'dec/step ms', round(p['decode_ms']/${TOKENS:-64},3), p)"
done
