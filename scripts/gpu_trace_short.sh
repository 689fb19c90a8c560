# kernel trace of a short full-size run (64 tokens); per-step kernel time accounting
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/trace -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --max-tokens 64 --no-cpu-baseline > gpurun_out/trace_bench.log 2>&1 || exit $?
grep '^{' gpurun_out/trace_bench.log | python -c "import json,sys; d=json.load(sys.stdin); print('RTF', d['value'], d['phase_ms'])"
