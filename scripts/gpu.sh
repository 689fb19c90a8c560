# One parameterised driver for every GPU-side measurement (run from the repo
# root on the GPU box, e.g.  gpurun -- bash scripts/gpu.sh suite bench).
# Tasks run in the order given; the first failure ends the call (no retries).
# Results land in gpurun_out/$OUT (default gpurun_out/run); the ones the docs
# cite are copied into profiles/ by hand.
#
#   suite           GPU parity suite (-m gpu, verbose prints) + smoke()
#   bench           default bench line                        -> bench.json
#   configs         BASELINE configs 2, 3, 5 (32 / 1 clip) and f16 precision
#   trace           kernel trace of the bench's decode (BENCH_ARGS; 24 tokens):
#                   tools/timeline.py, per-grid durations, in-graph xattn summary
#   layers          kernel trace of the one-clip decode -> layer_table.txt (per-launch table of one layer)
#   pmc             FETCH_SIZE / WRITE_SIZE passes -> pmc_traffic.json
#   stats           rocprofv3 --kernel-trace --stats of one bench step
#   gemm            encoder GEMM kernels A/B (tools/enc_ab.py, ROWS_LIST, MODES 0 tile / 5 wide) + MFMA PMC
#   gemmpmc         counter passes over the ring kernel and its timing builds
#   widestamps      the wide kernel's K-loop phases and in-kernel clock (stamp build)
#   gemmvariants    encoder-GEMM library variants in one process ($VARIANTS)
#   groups          bench at WA_DECODE_GROUPS in $GLIST
#   env             bench under each ';'-separated assignment list in $ENVLIST
#   libs            bench with library variants whisper-burn_amd/diag/<v>/$LIB ($VARIANTS)
#   round           suite, trace, pmc, stats, gemm, bench -- the round-end set
#
# Env: OUT (subdir), ROUND (tag), BENCH_ARGS (extra bench.py args).
set -o pipefail
O=gpurun_out/${OUT:-run}
R=${ROUND:-r03}
mkdir -p "$O"
export TMPDIR=/tmp
ROOT=$(pwd)

bench_line() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 600 python bench.py "$@" --json-out "$O/$n.json" > "$O/$n.log" 2>&1 || { tail -20 "$O/$n.log"; return 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['unit'], d['phase_ms'], 'xattn us', d['roofline_cross_attention']['avg_us'], 'q4 TF', d['roofline_q4_gemm']['achieved'])"
}

trace_csv() {  # dir -> the kernel_trace.csv rocprofv3 wrote under it
  ls "$1"/*/run_kernel_trace.csv "$1"/run_kernel_trace.csv 2>/dev/null | head -1
}

task_suite() {
  timeout -k 10 900 python -u -m pytest tests -q -m gpu -s --timeout 300 --timeout-method thread -rf > "$O/pytest_gpu.log" 2>&1
  local rc=$?
  grep -E "passed|failed|worst|tokens equal|FAILED" "$O/pytest_gpu.log" | tail -30
  [ $rc -eq 0 ] || return $rc
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || return 1
  tail -1 "$O/smoke.log"
}

task_bench() { bench_line bench $BENCH_ARGS; }

task_configs() {  # every line timed over 3 steps after 1 warmup
  local S="--steps 3 --warmup 1"
  bench_line c2_medium_b1 --variant medium --clips-per-gpu 1 --no-cpu-baseline $S || return 1
  bench_line c3_large_v3_b1 --clips-per-gpu 1 --no-cpu-baseline $S || return 1
  bench_line c5_large_v3_f16w --weights f16 --no-cpu-baseline $S || return 1
  bench_line c5_large_v3_f16w_b1 --weights f16 --clips-per-gpu 1 --no-cpu-baseline $S || return 1
  bench_line c4_precision_f16 --precision f16 --no-cpu-baseline $S
}

task_trace() {
  timeout -k 10 600 rocprofv3 --kernel-trace -d "$O/trace" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 \
    --max-tokens 24 --fixed-length --no-cpu-baseline $BENCH_ARGS > "$O/trace.log" 2>&1 || { tail "$O/trace.log"; return 1; }
  local f; f=$(trace_csv "$O/trace")
  python3 tools/timeline.py "$f" > "$O/timeline.txt" || return 1
  python3 scripts/trace_by_grid.py "$f" "skinny|q4_gemm_decode|xattn|dec_self|logits" "$O/chain_grid.json" > /dev/null || return 1
  python3 scripts/in_graph_summary.py "$O/chain_grid.json" large_v3 q4_0 f16x2 32 "$O/xattn_in_graph.json" || return 1
  python3 scripts/decode_overlap.py "$f" large_v3 q4_0 f16x2 32 "$O/decode_overlap.json" > "$O/decode_overlap.log" || return 1
  cat "$O/timeline.txt" "$O/decode_overlap.log"
  gzip -f "$f"
}

task_layers() {  # one-clip decode (BASELINE config 3): the per-launch table of one layer (tools/layer_table.py)
  timeout -k 10 600 rocprofv3 --kernel-trace -d "$O/ltrace" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 \
    --clips-per-gpu 1 --max-tokens 48 --fixed-length --no-cpu-baseline --seq-steps 0 > "$O/ltrace.log" 2>&1 || { tail "$O/ltrace.log"; return 1; }
  local f; f=$(trace_csv "$O/ltrace")
  python3 tools/layer_table.py "$f" "$O/layer_table.json" | tee "$O/layer_table.txt" || return 1
  gzip -f "$f"
}

task_pmc() {
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $C --kernel-include-regex "q4_gemm|xattn" -d "gpurun_out/pmc_${C}_$R" -o run --output-format csv \
      -- python3 bench.py --steps 1 --warmup 0 --max-tokens 8 --no-cpu-baseline $BENCH_ARGS > "$O/pmc_$C.log" 2>&1 || return 1
  done
  python3 scripts/pmc_summary.py $R "$O/pmc_traffic.json" > "$O/pmc_summary.log" || return 1
  rm -f gpurun_out/pmc_*_$R/*/run_counter_collection.csv gpurun_out/pmc_*_$R/run_counter_collection.csv
  tail -5 "$O/pmc_summary.log"
}

task_stats() {
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/stats" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 \
    --no-cpu-baseline $BENCH_ARGS --json-out "$O/bench_under_rocprof.json" > "$O/stats.log" 2>&1 || return 1
  cp "$(ls "$O"/stats/*/run_kernel_stats.csv "$O"/stats/run_kernel_stats.csv 2>/dev/null | head -1)" "$O/kernel_stats.csv"
  # the Q4 GEMM launches per queue: full width (what roofline_q4_gemm times) vs the CU-masked encoder stream
  python3 scripts/kernel_by_queue.py "$(trace_csv "$O/stats")" "q4_gemm_wide|q4_gemm_prefill|q4_gemm_enc" \
    "$O/q4_gemm_by_queue.json" | tee "$O/q4_gemm_by_queue.txt" || return 1
  rm -f "$(trace_csv "$O/stats")"
  python3 scripts/kstats.py "$O/kernel_stats.csv" 20
}

task_gemm() {
  for r in ${ROWS_LIST:-1500 48000}; do
    ROWS=$r MODES=${MODES:-0,5} timeout -k 10 300 python -u tools/enc_ab.py > "$O/enc_ab_$r.log" 2>&1 || return 1
    grep -v amdgpu.ids "$O/enc_ab_$r.log"
  done
  cd /tmp
  ROWS=48000 MODES=0,5 ROUNDS=1 REPS=2 timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
    SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-include-regex "prefill|q4_gemm_enc|wide" \
    -d "$ROOT/$O/gemm_pmc" -o run --output-format csv -- python3 "$ROOT/tools/enc_ab.py" > "$ROOT/$O/gemm_pmc.log" 2>&1 || { cd "$ROOT"; return 1; }
  cd "$ROOT"
  python3 scripts/mfma_summary.py "$O/gemm_pmc" | tee "$O/q4_gemm_mfma.txt"
}

# Counter passes over the encoder ring kernel (L geometry, M = 48000) for the
# product and the encdiag timing builds (1: no scale FMAs, 2: + no dequant):
# which unit bounds it.  Counters not listed by `rocprofv3 -L` are dropped.
task_gemmpmc() {
  cd /tmp
  timeout -s KILL 60 rocprofv3 -L > "$ROOT/$O/counters.txt" 2>&1
  local avail; avail=$(grep -oE "\bSQ_[A-Z0-9_]+|\bGRBM_[A-Z0-9_]+|\bTCP_[A-Z0-9_]+" "$ROOT/$O/counters.txt" | sort -u)
  local P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
  local P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
  for V in base ${ENCDIAGS:-1 2}; do
    local LD=""; [ "$V" = base ] || LD="$ROOT/whisper-burn_amd/encdiag/$V"
    local i=0
    for P in "$P1" "$P2"; do
      i=$((i + 1))
      local C=""; for c in $P; do echo "$avail" | grep -qx "$c" && C="$C $c"; done
      echo "variant $V pass $i:$C"
      WQ4_LIB_DIR=$LD ROWS=48000 MODES=${GMODE:-2} ROUNDS=1 REPS=3 timeout -s KILL 120 rocprofv3 --pmc $C \
        --kernel-include-regex "q4_gemm_enc|prefill" -d "$ROOT/$O/gpmc_${V}_$i" -o run --output-format csv \
        -- python3 "$ROOT/tools/enc_ab.py" > "$ROOT/$O/gpmc_${V}_$i.log" 2>&1 || { cd "$ROOT"; return 1; }
      python3 "$ROOT/scripts/mfma_summary.py" "$ROOT/$O/gpmc_${V}_$i" raw | tee -a "$ROOT/$O/gemm_counters.txt"
    done
  done
  cd "$ROOT"
}

# The wide kernel's K-loop phases (s_memtime / s_memrealtime stamps of
# waves 0 and 4 per workgroup: vmcnt, barrier, LDS-DMA issue, compute, and
# the in-kernel clock).  Needs the stamp build:
#   make -C whisper-burn_amd variant V=stampw DEFS=-DWQ4_WIDE_STAMP=1
task_widestamps() {
  WQ4_LIB_DIR=whisper-burn_amd/diag/stampw timeout -k 10 300 python -u tools/wide_stamps.py > "$O/wide_stamps.log" 2>&1 || return 1
  grep -v amdgpu.ids "$O/wide_stamps.log"
}

# Encoder-GEMM library variants timed in one process (tools/pf_variants.py):
# lib/libwq4.so against whisper-burn_amd/diag/<v>/libwq4.so for v in
# $VARIANTS (make -C whisper-burn_amd variant V=<v> DEFS=...), kernel mode
# $ENC_MODE (5: the wide kernel), bit identity against the product reported.
task_gemmvariants() {
  local libs="whisper-burn_amd/lib/libwq4.so"
  for v in $VARIANTS; do libs="$libs whisper-burn_amd/diag/$v/libwq4.so"; done
  ENC_MODE=${ENC_MODE:-5} ROUNDS=${ROUNDS:-4} timeout -k 10 500 python -u tools/pf_variants.py $libs > "$O/gemm_variants.log" 2>&1 || return 1
  grep -v amdgpu.ids "$O/gemm_variants.log"
}

task_groups() {
  for G in ${GLIST:-1 2 3}; do
    WA_DECODE_GROUPS=$G bench_line groups_$G --no-cpu-baseline $BENCH_ARGS || return 1
  done
}

task_env() {
  local i=0
  IFS=';' read -ra RUNS <<< "$ENVLIST"
  for E in "${RUNS[@]}"; do
    i=$((i + 1))
    echo "env $i: $E"
    ( export $E; bench_line env_$i --no-cpu-baseline $BENCH_ARGS ) || return 1
  done
}

task_libs() {  # variants load from their own directory (WQ4_LIB_DIR); lib/ is never touched
  for V in base ${VARIANTS} base; do
    if [ "$V" = base ]; then
      bench_line lib_$V --no-cpu-baseline $BENCH_ARGS || return 1
    else
      [ -f whisper-burn_amd/diag/$V/libwq4.so ] && [ -f whisper-burn_amd/diag/$V/libwhisper_amd.so ] || { echo "diag/$V incomplete"; return 1; }
      WQ4_LIB_DIR=$ROOT/whisper-burn_amd/diag/$V bench_line lib_$V --no-cpu-baseline $BENCH_ARGS || return 1
    fi
  done
}

task_round() {
  task_suite && task_trace && task_pmc && task_stats && task_gemm && task_bench
}

[ $# -gt 0 ] || { sed -n 2,24p "$0"; exit 2; }
for t in "$@"; do
  echo "== $t"
  "task_$t" || { echo "task $t failed"; exit 1; }
done
