# One clip (BASELINE config 3): decode with the LayerNorm-fold GEMMs on the
# 8-wave decode kernel (policy 0, the model's choice) vs the decode-step
# kernel (policy 3; note policy 3 also moves the encoder GEMMs).
mkdir -p gpurun_out
export TMPDIR=/tmp
for pol in 0 3; do
  timeout -k 10 300 python -c "
import sys; sys.argv = ['bench.py', '--clips-per-gpu', '1', '--no-cpu-baseline', '--json-out', 'gpurun_out/pol$pol.json']
sys.path.insert(0, 'whisper-burn_amd'); import wq4; wq4.set_kernel_policy($pol); import bench; bench.main()" > gpurun_out/pol$pol.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/pol$pol.json')); print('policy $pol', d['value'], d['phase_ms'])"
done
