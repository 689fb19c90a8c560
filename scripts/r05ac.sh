# xattn frame splits S = 6 / 7 against 8 (product) at 32 clips, sequential
set -o pipefail
O=gpurun_out/r05ac; mkdir -p $O; export TMPDIR=/tmp
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --sequential --fixed-length --steps 5 --warmup 2 --json-out $O/$n.json > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); p=d['phase_ms']; print('$n', d['value'], round(p['decode_ms'],1))"
}
run s8 A=1 && run s6 WQ4_LIB_DIR=whisper-burn_amd/diag/s6 && run s7 WQ4_LIB_DIR=whisper-burn_amd/diag/s7 && run s8b A=1
