# HIP runtime knobs against the dependent-launch floor and the decode:
# graph chain floor and sequential bench (10 steps) per setting
set -o pipefail
O=gpurun_out/r05aa; mkdir -p $O; export TMPDIR=/tmp
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 120 python3 scripts/chain_floor.py > $O/$n.chain.log 2>&1 || { tail -3 $O/$n.chain.log; return 1; }
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --sequential --steps 10 --warmup 3 --json-out $O/$n.json > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['phase_ms'])"; tail -1 $O/$n.chain.log
}
run base A=1 && run devkarg HIP_FORCE_DEV_KERNARG=1 && run nodevkarg HIP_FORCE_DEV_KERNARG=0 && run nocapture DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 && run nohdp DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0 && run base2 A=1
