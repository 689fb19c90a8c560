set -o pipefail
O=gpurun_out/${OUT:-r06f}; mkdir -p $O
WQ4_LIB_DIR=whisper-burn_amd/diag/stampw timeout -k 10 300 python -u tools/wide_stamps.py > $O/stamps.log 2>&1; rc=$?; cat $O/stamps.log; exit $rc
