# PMC passes on the isolated cross-attention kernels (variant $V), one counter group per pass
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-2}
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  WA_XATTN_MAIN=$V timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex xattn_main -d gpurun_out/pmc_x$i -o run --output-format csv -- python3 whisper-burn_amd/tools/xattn_bench.py --clips 32 --iters 5 > gpurun_out/pmc_x$i.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for f in glob.glob("gpurun_out/pmc_x*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:28s} {sum(v) / len(v):14.0f}")
PY
rm -f gpurun_out/pmc_x*/run_counter_collection.csv
