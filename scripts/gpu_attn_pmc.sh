# Encoder attention counters (MFMA busy, wave states, VALU count) from a short bench run.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-include-regex "encoder_attention|conv_gelu|layernorm" -d gpurun_out/attn_pmc -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --max-tokens 4 --no-cpu-baseline > gpurun_out/attn_pmc.log 2>&1 || exit $?
python3 scripts/mfma_summary.py gpurun_out/attn_pmc
python3 scripts/mfma_summary.py gpurun_out/attn_pmc raw
rm -f gpurun_out/attn_pmc/*/run_counter_collection.csv gpurun_out/attn_pmc/run_counter_collection.csv
