# HIP hardware queues per process: 4 (default) against 3 / 2, pipelined and
# sequential bench, 10 steps
set -o pipefail
O=gpurun_out/r05ai; mkdir -p $O; export TMPDIR=/tmp
run() {  # name, env, args...
  local n=$1 e=$2; shift 2
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 --json-out $O/$n.json "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; return 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['phase_ms'])"
}
run q4 A=1 && run q3 GPU_MAX_HW_QUEUES=3 && run q2 GPU_MAX_HW_QUEUES=2 && run q3s GPU_MAX_HW_QUEUES=3 --sequential && run q2s GPU_MAX_HW_QUEUES=2 --sequential && run q4s A=1 --sequential
