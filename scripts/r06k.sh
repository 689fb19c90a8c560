# round 6: wide-kernel setprio / v_and_or A/B (bit identity + timings)
set -o pipefail
O=gpurun_out/${OUT:-r06k}; mkdir -p $O
L=whisper-burn_amd
ENC_MODE=5 ROUNDS=4 timeout -k 10 500 python -u tools/pf_variants.py $L/lib/libwq4.so $L/diag/prio/libwq4.so $L/diag/andor/libwq4.so $L/diag/both/libwq4.so > $O/variants.log 2>&1 || { tail $O/variants.log; exit 1; }
cat $O/variants.log
