# round 6: wide-kernel diagnostics -- variant timings + PMC on the tile and wide kernels
set -o pipefail
O=gpurun_out/${OUT:-r06b}; mkdir -p $O
ROOT=$(pwd); export TMPDIR=/tmp
L=whisper-burn_amd
ENC_MODE=5 ROUNDS=3 timeout -k 10 300 python -u tools/pf_variants.py $L/lib/libwq4.so $L/diag/wide1/libwq4.so $L/diag/wide2/libwq4.so > $O/variants_wide.log 2>&1 || { tail $O/variants_wide.log; exit 1; }
cat $O/variants_wide.log
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
cd /tmp
for MODE in 0 5; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i + 1))
    ROWS=48000 MODES=$MODE ROUNDS=1 REPS=3 timeout -s KILL 120 rocprofv3 --pmc $P \
      --kernel-include-regex "prefill|wide" -d "$ROOT/$O/pmc_${MODE}_$i" -o run --output-format csv \
      -- python3 "$ROOT/tools/enc_ab.py" > "$ROOT/$O/pmc_${MODE}_$i.log" 2>&1 || { tail "$ROOT/$O/pmc_${MODE}_$i.log"; exit 1; }
    python3 "$ROOT/scripts/mfma_summary.py" "$ROOT/$O/pmc_${MODE}_$i" raw >> "$ROOT/$O/gemm_counters.txt"; python3 "$ROOT/scripts/mfma_summary.py" "$ROOT/$O/pmc_${MODE}_$i"
  done
done
