# Bench RTF with xattn_out at 2 rows per workgroup for <= 16 rows (a build with that rule)
# vs 4 (WA_XATTN_OUT_ROWS=4 build in whisper-burn_amd/diag/or4), alternating; r02: 2 rows slower.
mkdir -p gpurun_out
export TMPDIR=/tmp
cp whisper-burn_amd/lib/libwhisper_amd.so /tmp/libwa.base
for V in base or4 base or4; do
  if [ $V = base ]; then cp /tmp/libwa.base whisper-burn_amd/lib/libwhisper_amd.so; else cp whisper-burn_amd/diag/or4/libwhisper_amd.so whisper-burn_amd/lib/libwhisper_amd.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --json-out gpurun_out/bench_$V.json > gpurun_out/bench_$V.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_$V.json')); print('$V', d['value'], d['phase_ms'])"
done
cp /tmp/libwa.base whisper-burn_amd/lib/libwhisper_amd.so
