# Round 3, call D: full GPU suite (regression after the ring kernel), then
# one-clip / few-clip A/B of the encoder GEMM kernels.
set -o pipefail
mkdir -p gpurun_out/r03d
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03d/tests.log 2>&1 || { tail -40 gpurun_out/r03d/tests.log; exit 1; }
tail -3 gpurun_out/r03d/tests.log
for r in 1500 3000 6000 12000; do
  MODES=0,3,4 ROWS=$r ROUNDS=7 timeout -k 10 240 python -u tools/enc_ab.py > gpurun_out/r03d/ab$r.log 2>&1 || exit 1
done
cat gpurun_out/r03d/ab*.log | grep -v amdgpu.ids
