# Decode groups x hardware queues: does a 3rd/4th decode group pay once each
# group's stream has its own hardware queue (GPU_MAX_HW_QUEUES, default 4)?
mkdir -p gpurun_out
for Q in 4 8; do
  for G in 2 3 4; do
    GPU_MAX_HW_QUEUES=$Q WA_DECODE_GROUPS=$G timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline \
      --json-out gpurun_out/hwq_${Q}_g${G}.json > gpurun_out/hwq_${Q}_g${G}.log 2>&1 || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/hwq_${Q}_g${G}.json')); print('hwq $Q groups $G', d['value'], d['phase_ms'])"
  done
done
