# PMC passes for one kernel family ($KRX regex) in a short bench run (2 tokens)
mkdir -p gpurun_out
export TMPDIR=/tmp
KRX=${KRX:-encoder_attention}
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "$KRX" -d gpurun_out/pmc_k$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --max-tokens 2 --fixed-length --no-cpu-baseline > gpurun_out/pmc_k$i.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for f in glob.glob("gpurun_out/pmc_k*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:28s} {sum(v) / len(v):16.0f}  (n={len(v)})")
PY
rm -f gpurun_out/pmc_k*/run_counter_collection.csv
