# encoder GEMM kernels on the pipelined transcribe's 32-CU masked stream
set -o pipefail
O=gpurun_out/r05r2; mkdir -p $O; export TMPDIR=/tmp
MASK_CUS=32 ROWS=48000 MODES=0,2,3 ROUNDS=3 REPS=2 timeout -k 10 400 python -u tools/enc_ab.py 2>&1 | grep -v amdgpu.ids | tee $O/enc_ab_mask32.log
