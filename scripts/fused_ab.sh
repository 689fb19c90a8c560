# A/B of the decode step's in-launch projections (bench.py --fused-proj mask):
# 0 none, 1 self-attention q/k/v (one workgroup per head), 2 cross-attention
# query, 4 with 1: the self-attention projection over 8 workgroups per head
set -o pipefail
O=gpurun_out/${AB_OUT:-r05a}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_fused_decode_gpu.py -x -v --timeout 300 --timeout-method thread > $O/fused.log 2>&1 || { grep -E "PASS|FAIL|Error" $O/fused.log | head -20; exit 1; }
grep -cE "PASSED" $O/fused.log
for F in 0 2 5 7 3; do
  timeout -k 10 300 python bench.py --clips-per-gpu 1 --no-cpu-baseline --fused-proj $F --json-out $O/c1_$F.json > $O/c1_$F.log 2>&1 || exit 1
  python3 -c "import json; d=json.load(open('$O/c1_$F.json')); print('1clip mask $F', d['value'], d['phase_ms'])"
done
for F in 0 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --fused-proj $F --json-out $O/c32_$F.json > $O/c32_$F.log 2>&1 || exit 1
  python3 -c "import json; d=json.load(open('$O/c32_$F.json')); print('32clip mask $F', d['value'], d['phase_ms'])"
done
for F in 0 7; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/st_$F -o run --output-format csv -- python3 bench.py --clips-per-gpu 1 --steps 1 --warmup 1 --max-tokens 64 --fixed-length --no-cpu-baseline --fused-proj $F > $O/st_$F.log 2>&1 || exit 1
  f=$(ls $O/st_$F/*/run_kernel_stats.csv $O/st_$F/run_kernel_stats.csv 2>/dev/null | head -1); cp $f $O/kstats_$F.csv
  python3 scripts/kstats.py $O/kstats_$F.csv 14
  rm -f $(ls $O/st_$F/*/run_kernel_trace.csv $O/st_$F/run_kernel_trace.csv 2>/dev/null)
done
