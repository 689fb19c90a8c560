# Cross-attention kernels in isolation (tools/xattn_micro.hip), one binary per
# WA_XATTN_DIAG attribution variant (XDIAGS) + any extra -D variants in
# XVARIANTS ("name:flags" items); each binary runs with the split-phase path
# off (WA_XATTN_SMALL_ROWS=0) and on for up to 8 rows.
# Build here: XBUILD=1 sh scripts/xattn_micro.sh; run on the GPU box:
# sh scripts/xattn_micro.sh
set -e
OUT=whisper-burn_amd/build/xmicro
if [ -n "$XBUILD" ]; then
  mkdir -p $OUT
  for d in ${XDIAGS:-0}; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude -DWA_XATTN_DIAG=$d \
      whisper-burn_amd/tools/xattn_micro.hip -o $OUT/diag$d &
  done
  for v in $XVARIANTS; do
    n=${v%%:*}; f=$(echo ${v#*:} | tr ',' ' ')
    /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude $f \
      whisper-burn_amd/tools/xattn_micro.hip -o $OUT/v_$n &
  done
  wait
  exit 0
fi
mkdir -p gpurun_out
for b in $OUT/*; do
  for sr in 0 8; do
    echo "== $(basename $b) WA_XATTN_SMALL_ROWS=$sr"
    WA_XATTN_SMALL_ROWS=$sr timeout -k 10 60 $b 200
  done
done 2>&1 | tee gpurun_out/xattn_micro.log
