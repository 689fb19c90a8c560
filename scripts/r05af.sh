# xattn frame splits 7 / 6 in the PIPELINED transcribe: 16 x S main workgroups
# per group against the 28 CUs per XCD the 32-CU encoder mask leaves free
set -o pipefail
O=gpurun_out/r05af; mkdir -p $O; export TMPDIR=/tmp
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 --json-out $O/$n.json > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); p=d['phase_ms']; print('$n', d['value'], p, d['pipeline']['overlap_layers'], round(d['pipeline']['masked_ms'],1))"
}
run s8 A=1 && run s7 WQ4_LIB_DIR=whisper-burn_amd/diag/s7 && run s6 WQ4_LIB_DIR=whisper-burn_amd/diag/s6 && run s7f100 WQ4_LIB_DIR=whisper-burn_amd/diag/s7 WA_ENC_FILL=1.0 && run s8b A=1
