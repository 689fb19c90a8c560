# log-mel front-end: GPU parity tests, then a short audio->tokens bench and a kernel-trace profile of it
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_mel_gpu.py -q -m gpu -x > gpurun_out/pytest_mel.log 2>&1; rc=$?
echo "pytest mel rc=$rc"; tail -5 gpurun_out/pytest_mel.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --audio --steps 2 --warmup 1 --max-tokens 32 --fixed-length --no-cpu-baseline \
  --json-out gpurun_out/bench_audio.json > gpurun_out/bench_audio.log 2>&1 || exit $?
cat gpurun_out/bench_audio.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mel -o run --output-format csv -- \
  python3 bench.py --audio --steps 1 --warmup 1 --max-tokens 8 --fixed-length --no-cpu-baseline \
  > gpurun_out/prof_mel.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/prof_mel/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "mel" in r["Name"]:
            print(r["Name"][:60], r["Calls"], r["AverageNs"])
PY
