# One-clip configs (BASELINE configs 3 and 2) with the cross-attention split
# phases off (WA_XATTN_SMALL_ROWS=0, the fused kernel) and on (default).
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, small-rows, bench args
  local n=$1 sr=$2; shift 2
  WA_XATTN_SMALL_ROWS=$sr timeout -k 10 300 python bench.py --no-cpu-baseline --json-out gpurun_out/sr_${n}_$sr.json "$@" > gpurun_out/sr_${n}_$sr.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/sr_${n}_$sr.json')); print('$n small_rows=$sr', d['value'], d['unit'], d['phase_ms'])"
}
run c3_large_v3_b1 0 --clips-per-gpu 1
run c3_large_v3_b1 4 --clips-per-gpu 1
run c2_medium_b1 0 --variant medium --clips-per-gpu 1
run c2_medium_b1 4 --variant medium --clips-per-gpu 1
