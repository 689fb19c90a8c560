# Decode-GEMM timing diagnostics: the one-group 32-clip chain trace with the
# product libwq4 and with each WQ4_DIAG variant (wrong results, timing only).
mkdir -p gpurun_out
export TMPDIR=/tmp
for V in 0 ${DIAGS:-1 2 3 4}; do
  if [ "$V" = 0 ]; then unset WQ4_LIB_DIR; else export WQ4_LIB_DIR=$PWD/whisper-burn_amd/diag/$V; fi
  WA_DECODE_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/diag_$V -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --max-tokens 16 --fixed-length --no-cpu-baseline > gpurun_out/diag_$V.log 2>&1 || exit $?
  f=$(ls gpurun_out/diag_$V/*/run_kernel_trace.csv gpurun_out/diag_$V/run_kernel_trace.csv 2>/dev/null | head -1)
  echo "== variant $V"
  python3 scripts/trace_gaps.py $f | grep -E "q4_gemm_decode|decode kernels"
  rm -f $f
done
