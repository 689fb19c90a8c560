# Round-5 measurement set at HEAD (run on the GPU box from the repo root):
# range-guard + model parity spot check, limb microbenchmark, then the
# gpu.sh trace / pmc / gemmpmc tasks whose outputs feed bench.py's roofline.
set -o pipefail
O=gpurun_out/r05b; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_range_guard.py tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/limb_micro > $O/limb.log 2>&1 || exit 1
cat $O/limb.log
OUT=r05b ROUND=r05 bash scripts/gpu.sh trace pmc gemmpmc
