# GPU suite + smoke, then the default bench line (no chain trace).
bash scripts/gpu_suite.sh || exit $?
timeout -k 10 600 python bench.py --json-out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); print('RTF', d['value'], d['phase_ms'], 'xattn', d['roofline_cross_attention']['avg_us'], 'q4', d['roofline_q4_gemm'])"
