# kernel-trace of the cross-attention kernels in isolation (Large-V3 decode shape, 32 clips)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_xattn -o run --output-format csv -- \
  python3 whisper-burn_amd/tools/xattn_bench.py --clips 32 --iters 20 $XARGS > gpurun_out/prof_xattn.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/prof_xattn/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
