# Decode-step iteration without the test suite: stamped GEMM phases and the
# per-grid kernel trace at the bench's own grouping (2 groups of 16 clips
# unless GROUPS_N says otherwise), then the bench line.
G=${GROUPS_N:-2}
WA_DECODE_GROUPS=$G WQ4_LIB_DIR=$PWD/whisper-burn_amd/diag/stamp timeout -k 10 300 python scripts/skinny_stamps.py 2>&1 | grep -v amdgpu.ids || exit $?
GROUPS_N=$G ROUND=${ROUND:-r02} bash scripts/gpu_chain_trace.sh || exit $?
timeout -k 10 600 python bench.py --no-cpu-baseline --json-out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); print('RTF', d['value'], d['phase_ms'])"
