# Round-5 final set at HEAD (after the epilogue / GELU / fill changes): GPU
# suite + smoke, decode trace and PMC traffic (copied into profiles/ before
# the bench reads them), kernel stats, then the bench at the driver's counts
# (pipelined and --sequential).
set -o pipefail
export OUT=r05fin ROUND=r05fin
O=gpurun_out/$OUT
bash scripts/gpu.sh suite trace pmc stats || exit 1
cp $O/decode_overlap.json $O/xattn_in_graph.json $O/pmc_traffic.json profiles/ || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --json-out $O/bench20.json > $O/bench20.log 2>&1 || { tail -5 $O/bench20.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench20.json')); print('pipe20', d['value'], d['phase_ms'], d['roofline']['frac'])"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --sequential --no-cpu-baseline --json-out $O/seq20.json > $O/seq20.log 2>&1 || { tail -5 $O/seq20.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/seq20.json')); print('seq20', d['value'], d['phase_ms'])"
