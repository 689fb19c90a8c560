set -o pipefail
O=gpurun_out/${OUT:-r06a}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_q4_gpu.py -x -q -k "enc_kernel_bit_identical or headmajor_ring" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
ROWS=48000 MODES=0,5 ROUNDS=5 timeout -k 10 300 python -u tools/enc_ab.py > $O/enc_ab.log 2>&1; rc=$?; cat $O/enc_ab.log; exit $rc
