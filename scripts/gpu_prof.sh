# rocprofv3 kernel trace of a short bench run (stats summary -> gpurun_out/prof_*)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --clips-per-gpu ${CLIPS:-32} --steps 1 --warmup 1 --max-tokens ${TOKENS:-32} --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || exit $?
tail -1 gpurun_out/prof_bench.log
find gpurun_out/prof -name "*stats*" | head
