# Bench RTF (two decode groups) at 1-4 hardware queues per process (GPU_MAX_HW_QUEUES; the box default is 4).
mkdir -p gpurun_out
for Q in 4 2 3 1 4; do
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline \
    --json-out gpurun_out/hwq_$Q.json > gpurun_out/hwq_$Q.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/hwq_$Q.json')); print('hwq $Q', d['value'], d['phase_ms'])"
done
