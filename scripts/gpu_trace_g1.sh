# kernel trace of a short G=1 decode (per-kernel durations and gaps inside one step)
mkdir -p gpurun_out
export TMPDIR=/tmp
WA_DECODE_GROUPS=${G:-1} timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_g1 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --max-tokens 32 --fixed-length --no-cpu-baseline > gpurun_out/trace_g1.log 2>&1 || exit $?
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/trace_g1/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# keep the last 3000 dispatches (inside the timed decode loop)
tail = rows[-3000:]
with open("gpurun_out/trace_g1/tail.csv", "w") as f:
    w = csv.writer(f)
    w.writerow(["name", "start", "end", "queue"])
    for r in tail:
        w.writerow([r["Kernel_Name"][:60], r["Start_Timestamp"], r["End_Timestamp"], r.get("Queue_Id", "")])
PY
rm -f gpurun_out/trace_g1/run_kernel_trace.csv
