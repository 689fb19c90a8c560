# kernel trace of a short decode (per-kernel durations inside one step); env passes through
mkdir -p gpurun_out
export TMPDIR=/tmp
WA_DECODE_GROUPS=${G:-1} timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/trace_g1 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --max-tokens 32 --fixed-length --no-cpu-baseline --clips-per-gpu ${CLIPS:-32} > gpurun_out/trace_g1.log 2>&1 || exit $?
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/trace_g1/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
with open("gpurun_out/trace_g1/tail.csv", "w") as f:
    w = csv.writer(f)
    w.writerow(["name", "start", "end"])
    for r in rows[-3000:]:
        w.writerow([r["Kernel_Name"][:60], r["Start_Timestamp"], r["End_Timestamp"]])
PY
rm -f gpurun_out/trace_g1/run_kernel_trace.csv
python3 scripts/step_profile.py gpurun_out/trace_g1/tail.csv
