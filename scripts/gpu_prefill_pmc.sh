# prefill Q4 GEMM at the encoder fc1 shape: timing + PMC passes
mkdir -p gpurun_out
export TMPDIR=/tmp
SHAPE=${SHAPE:-48000,5120,1280}
timeout -k 10 120 python whisper-burn_amd/tools/q4_bench.py --shape $SHAPE --iters 5 --prec ${PREC:-0}
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex prefill -d gpurun_out/pmc_p$i -o run --output-format csv -- python3 whisper-burn_amd/tools/q4_bench.py --shape $SHAPE --iters 2 --no-graph --prec ${PREC:-0} > gpurun_out/pmc_p$i.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for f in glob.glob("gpurun_out/pmc_p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:28s} {sum(v) / len(v):14.0f}  (n={len(v)})")
PY
rm -f gpurun_out/pmc_p*/run_counter_collection.csv
