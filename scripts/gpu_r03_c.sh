# Round 3, call C: ring-kernel ablations (no scale FMAs; + no dequant) and PMC.
set -o pipefail
mkdir -p gpurun_out/r03c
export TMPDIR=/tmp
L="whisper-burn_amd/lib/libwq4.so whisper-burn_amd/encdiag/1/libwq4.so whisper-burn_amd/encdiag/2/libwq4.so"
for g in 2 3; do
  ENC_MODE=$g ROWS=48000 timeout -k 10 240 python -u tools/pf_variants.py $L > gpurun_out/r03c/abl_g$g.log 2>&1 || { cat gpurun_out/r03c/abl_g$g.log; exit 1; }
done
cat gpurun_out/r03c/abl_g2.log gpurun_out/r03c/abl_g3.log
cd /tmp
export MODES=2 ROWS=48000 ROUNDS=1 REPS=2
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-include-regex q4_gemm_enc -d $GRAFT_REPO_ROOT/gpurun_out/r03c/pmc1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/enc_ab.py > $GRAFT_REPO_ROOT/gpurun_out/r03c/pmc1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex q4_gemm_enc -d $GRAFT_REPO_ROOT/gpurun_out/r03c/pmc2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/enc_ab.py > $GRAFT_REPO_ROOT/gpurun_out/r03c/pmc2.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python3 scripts/mfma_summary.py gpurun_out/r03c/pmc1
python3 scripts/mfma_summary.py gpurun_out/r03c/pmc2 raw
