# Iteration loop for the decode step: GPU suite, stamped phase timing of the
# decode-step GEMM, bench line, one-group chain trace.
bash scripts/gpu_suite.sh || exit $?
WA_DECODE_GROUPS=1 WQ4_LIB_DIR=$PWD/whisper-burn_amd/diag/stamp timeout -k 10 300 python scripts/skinny_stamps.py 2>&1 | grep -v amdgpu.ids || exit $?
timeout -k 10 600 python bench.py --no-cpu-baseline --json-out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); print('RTF', d['value'], d['phase_ms'])"
ROUND=${ROUND:-r02} bash scripts/gpu_chain_trace.sh
