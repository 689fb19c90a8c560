# Bench RTF with library variants (whisper-burn_amd/diag/<variant>/<LIB>,
# tuning builds) swapped over the product build, product first and last.
LIB=${LIB:-libwq4.so}
cp whisper-burn_amd/lib/$LIB /tmp/$LIB.base
for V in base ${VARIANTS} base; do
  if [ "$V" = base ]; then cp /tmp/$LIB.base whisper-burn_amd/lib/$LIB; else cp whisper-burn_amd/diag/$V/$LIB whisper-burn_amd/lib/$LIB; fi
  timeout -k 10 400 python bench.py --no-cpu-baseline $BENCH_ARGS --json-out gpurun_out/bench_v$V.json > gpurun_out/bench_v$V.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_v$V.json')); print('$V RTF', d['value'], d['phase_ms'], 'xattn', d['roofline_cross_attention']['avg_us'])"
done
