# Encoder Q4 GEMM: kernel trace stats + PMC passes (MFMA busy / wave states;
# LDS and instruction counts), for POLICY (0 = block-scaled, 4 = f16-pair).
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUND:-r02}p${POLICY:-0}
timeout -k 10 300 python scripts/gemm_probe.py || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/gemm_$R -o run --output-format csv -- python3 scripts/gemm_probe.py > gpurun_out/gemm_$R.log 2>&1 || exit $?
f=$(ls gpurun_out/gemm_$R/*/run_kernel_stats.csv gpurun_out/gemm_$R/run_kernel_stats.csv 2>/dev/null | head -1)
cut -d, -f1-4 $f | grep -i prefill
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-include-regex prefill -d gpurun_out/gemm_pmc_$R -o run --output-format csv -- python3 scripts/gemm_probe.py > gpurun_out/gemm_pmc_$R.log 2>&1 || exit $?
python3 scripts/mfma_summary.py gpurun_out/gemm_pmc_$R
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex prefill -d gpurun_out/gemm_pmc2_$R -o run --output-format csv -- python3 scripts/gemm_probe.py > gpurun_out/gemm_pmc2_$R.log 2>&1 || exit $?
python3 scripts/mfma_summary.py gpurun_out/gemm_pmc2_$R raw
