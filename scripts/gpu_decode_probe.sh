# Decode-size Q4 GEMMs (ROWS rows) under the decode (2) and decode-step (3)
# kernels: per-kernel durations from a kernel trace.
mkdir -p gpurun_out
export TMPDIR=/tmp
for P in 2 3; do
  ROWS=${ROWS:-16} REPS=50 POLICY=$P timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/dprobe_p$P -o run --output-format csv -- python3 scripts/gemm_probe.py > gpurun_out/dprobe_p$P.log 2>&1 || exit $?
  f=$(ls gpurun_out/dprobe_p$P/*/run_kernel_trace.csv gpurun_out/dprobe_p$P/run_kernel_trace.csv 2>/dev/null | head -1)
  python3 scripts/trace_by_grid.py $f "q4_gemm_decode|skinny" gpurun_out/dprobe_grid_p$P.json
  rm -f $f
done
