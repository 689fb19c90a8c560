# round 6: tile (0) vs wide (5) encoder GEMM kernels, interleaved in one process, at several row counts
set -o pipefail
O=gpurun_out/${OUT:-r06g}; mkdir -p $O
for R in 48000 24000 12000 6000; do
  ROWS=$R MODES=0,5 ROUNDS=4 timeout -k 10 300 python -u tools/enc_ab.py > $O/enc_ab_$R.log 2>&1 || { tail $O/enc_ab_$R.log; exit 1; }
  grep TF $O/enc_ab_$R.log
done
