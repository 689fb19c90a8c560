# xattn kernels in isolation (Large-V3 decode shape, 32 clips), per WA_XATTN_MAIN variant in $VARS
mkdir -p gpurun_out
export TMPDIR=/tmp
for V in ${VARS:-0 1}; do
  WA_XATTN_MAIN=$V timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/px_$V -o run --output-format csv -- \
    python3 whisper-burn_amd/tools/xattn_bench.py --clips 32 --iters 20 > gpurun_out/px_$V.log 2>&1 || exit $?
  python3 - "$V" <<'PY'
import csv, glob, sys
for f in glob.glob(f"gpurun_out/px_{sys.argv[1]}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "xattn" in r["Name"]:
            print("variant", sys.argv[1], r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
  rm -f gpurun_out/px_$V/run_kernel_trace.csv
done
