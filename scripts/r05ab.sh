# is the 32-clip decode chain-bound or throughput-bound?  decode per step at
# 8 / 16 / 32 clips and 1 / 2 groups; 1 group also without graph packet
# capture (a 1.2 us longer dependent-launch floor)
set -o pipefail
O=gpurun_out/r05ab; mkdir -p $O; export TMPDIR=/tmp
run() {  # name, clips, env...
  local n=$1 c=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --sequential --fixed-length --steps 3 --warmup 1 --clips-per-gpu $c --json-out $O/$n.json > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); p=d['phase_ms']; print('$n', round(p['decode_ms'],1), 'ms decode,', round(p['decode_ms']/224*1e3,1), 'us/step')"
}
run c32g2 32 A=1 && run c32g1 32 WA_DECODE_GROUPS=1 && run c16g1 16 WA_DECODE_GROUPS=1 && run c16g2 16 WA_DECODE_GROUPS=2 && run c8g1 8 WA_DECODE_GROUPS=1 && run c16g1nc 16 WA_DECODE_GROUPS=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 && run c32g2nc 32 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
