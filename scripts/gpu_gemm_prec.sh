# Encoder Q4 GEMM probe at both precisions (f16x2 default, f16) + MFMA-busy PMC.
mkdir -p gpurun_out
export TMPDIR=/tmp
for P in 0 1; do
  PREC=$P timeout -k 10 300 python scripts/gemm_probe.py || exit $?
  PREC=$P timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-include-regex prefill -d gpurun_out/gemm_prec$P -o run --output-format csv -- python3 scripts/gemm_probe.py > gpurun_out/gemm_prec$P.log 2>&1 || exit $?
  python3 scripts/mfma_summary.py gpurun_out/gemm_prec$P
  rm -f gpurun_out/gemm_prec$P/*/run_counter_collection.csv gpurun_out/gemm_prec$P/run_counter_collection.csv
done
