# Cross-attention parity tests, then the bench line (RTF, cross-attention probe).
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "xattn or cross or full_size_tokens" --timeout 200 --timeout-method thread > gpurun_out/xq_tests.log 2>&1; rc=$?
tail -2 gpurun_out/xq_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline --json-out gpurun_out/bench_xq.json > gpurun_out/bench_xq.log 2>&1 || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_xq.json')); r=d['roofline_cross_attention']; print('RTF', d['value'], d['phase_ms'], 'xattn us', r['avg_us'], 'frac', r['frac'])"
