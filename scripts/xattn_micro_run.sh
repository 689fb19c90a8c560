mkdir -p gpurun_out/r05c
for b in whisper-burn_amd/build/xmicro/*; do
  echo "== $(basename $b)"
  WA_XATTN_SMALL_ROWS=0 timeout -k 10 60 $b 100 | grep main_us || exit 1
done 2>&1 | tee gpurun_out/r05c/xattn_micro.log
