# GPU parity tests, graph-timed decode GEMM shapes, then a profiled short model run
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python whisper-burn_amd/tools/q4_bench.py --decode-only --iters 50 > gpurun_out/q4_dec.log 2>&1 || exit $?
grep f16x2 gpurun_out/q4_dec.log
CLIPS=${CLIPS:-32} TOKENS=${TOKENS:-32} bash scripts/gpu_prof.sh
