# round 6: spread LDS-DMA issue -- bit identity, timings vs up-front issue, stamps
set -o pipefail
O=gpurun_out/${OUT:-r06e}; mkdir -p $O
L=whisper-burn_amd
timeout -k 10 300 python -u -m pytest tests/test_q4_gpu.py -x -q -k "enc_kernel_bit_identical or headmajor_ring" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
ENC_MODE=5 ROUNDS=3 timeout -k 10 400 python -u tools/pf_variants.py $L/lib/libwq4.so $L/diag/up/libwq4.so $L/diag/wide1/libwq4.so > $O/variants.log 2>&1 || { tail $O/variants.log; exit 1; }
cat $O/variants.log
WQ4_LIB_DIR=$L/diag/stampw timeout -k 10 300 python -u tools/wide_stamps.py > $O/stamps.log 2>&1; rc=$?; cat $O/stamps.log; exit $rc
