# A/B of env settings in ONE box (boxes differ by up to ~10%): "$AB" lines = env assignments per arm
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
while read -r ENVS; do
  i=$((i+1))
  env $ENVS timeout -k 10 300 python bench.py --steps 1 --warmup 1 --max-tokens ${TOKENS:-64} --fixed-length --no-cpu-baseline > gpurun_out/ab_$i.log 2>&1 || exit $?
  grep '^{' gpurun_out/ab_$i.log | python -c "import json,sys; d=json.load(sys.stdin); p=d['phase_ms']; print('[$ENVS] RTF', d['value'], 'dec/step ms', round(p['decode_ms']/${TOKENS:-64},3), 'enc', p['encoder_ms'])"
done <<< "$AB"
