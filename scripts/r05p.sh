# prefill GEMM: scalar scale FMAs (WQ4_PF_DIAG=3, -fno-slp-vectorize: bit-identical
# arithmetic) against the product's packed form, one process, interleaved.
set -o pipefail
O=gpurun_out/r05p; mkdir -p $O; export TMPDIR=/tmp
ROWS=48000 ROUNDS=5 REPS=5 timeout -k 10 300 python -u tools/pf_variants.py whisper-burn_amd/lib/libwq4.so whisper-burn_amd/pfdiag/3/libwq4.so 2>&1 | grep -v amdgpu.ids | tee $O/pf_variants.log
