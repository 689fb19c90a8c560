# Standalone logits + pick kernel durations (scripts/logits_probe.py).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for b in ${BS:-16 32}; do
  B=$b timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/lgp_$b -o run --output-format csv -- python3 scripts/logits_probe.py > gpurun_out/lgp_$b.log 2>&1 || exit $?
done
