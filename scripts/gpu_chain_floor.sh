# Dispatch floor of a chain of trivial dependent kernels (graph-replayed).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python scripts/chain_floor.py || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/floor -o run --output-format csv -- python3 scripts/chain_floor.py > gpurun_out/floor.log 2>&1 || exit $?
f=$(ls gpurun_out/floor/*/run_kernel_trace.csv gpurun_out/floor/run_kernel_trace.csv 2>/dev/null | head -1)
python3 scripts/trace_gaps.py $f gpurun_out/floor_gaps.json | head -8
rm -f $f
