# Bench RTF with cross-attention split-count variants against the product
# build.  Build the variants first (CPU side):
#   for S in 12 16; do hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DWA_XATTN_SPLITS=$S \
#     -c whisper-burn_amd/csrc/whisper/wa_xattn.hip -o whisper-burn_amd/build/wa_xattn_s$S.o && \
#     hipcc --offload-arch=gfx950 -shared -fPIC -o whisper-burn_amd/diag/xs$S/libwhisper_amd.so <the other
#     wa_*.o of whisper-burn_amd/build> whisper-burn_amd/build/wa_xattn_s$S.o -Lwhisper-burn_amd/lib -lwq4 \
#     -Wl,-rpath,'$ORIGIN'; done
cp whisper-burn_amd/lib/libwhisper_amd.so /tmp/libwhisper_amd.base.so
for V in base ${SPLITS:-12 16} base; do
  if [ "$V" = base ]; then cp /tmp/libwhisper_amd.base.so whisper-burn_amd/lib/libwhisper_amd.so; else cp whisper-burn_amd/diag/xs$V/libwhisper_amd.so whisper-burn_amd/lib/libwhisper_amd.so; fi
  timeout -k 10 400 python bench.py --no-cpu-baseline --json-out gpurun_out/bench_xs$V.json > gpurun_out/bench_xs$V.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_xs$V.json')); r=d['roofline_cross_attention']; print('splits $V RTF', d['value'], d['phase_ms']['decode_ms'], 'xattn us', r['avg_us'])"
done
