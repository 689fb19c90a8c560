#!/usr/bin/env python3
"""Benchmark: Whisper Large-V3 Q4_0 real-time factor on MI355X (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Both forms run N ranks: without a torch.distributed.run environment
(WORLD_SIZE unset) and N > 1, this process starts the N rank processes
itself (launch_ranks) before anything touches HIP, and exits with the first
failing rank's status.  `--dry-run` exercises the launch / rendezvous /
max-over-ranks logic with no GPU work (tests/test_bench_dist.py).

One "step" = one batch of synthetic 30-s clips transcribed end to end on each
GPU: conv front-end + 32-layer encoder + prompt + greedy KV-cached
decode (whisper.rs:51-128), mel already resident in HBM, token ids back on the
host.  Workload at N = 1: BASELINE.json config 4's per-GPU shard (32 clips of
the 256-clip / 8-GPU job); each rank runs its own clips (weak scaling, no
collective on the data path -- one process per GPU, independent replicas).
value = audio seconds of all ranks' clips / max-over-ranks wall seconds.

roofline: the dominant kernel by WALL time per step -- for the decode
cross-attention its summed GPU time scaled by the union / sum of its launch
intervals in the committed kernel trace (profiles/decode_overlap.json: the two
decode groups' launches overlap), for the serial encoder GEMMs their GPU time
-- the Q4 GEMMs (north-star
kernel, MFMA tile kernel, timed live with HIP events on their launch stream
during the timed steps; algorithmic FLOPs = 2*M*N*K per launch) or the decode
step's cross-attention (HBM stream of every clip's encoder output, f16 hi/lo
planes, shared by all heads -- no per-layer K/V caches; algorithmic bytes =
encoder planes + raw Wk, Wv + operands).  The cross-attention is HIP-event
timed by wa_probe_kernels right after the timed steps at the shape the decode
graphs run it (one decode group's clips, wa_decode_group_rows), and carries
the in-graph durations of the same grids from the committed rocprofv3 chain
trace (profiles/xattn_in_graph.json, scripts/in_graph_summary.py) as a
cross-check.  Both, and the decode-step fc1 GEMM, are reported.

cpu_baseline: the reference's CPU dequant->GEMM path
(src/gguf/tests.rs:60-87,172-184, restated in oracle/q4_oracle.c) on
Q4Linear 1280x1280 and Q4FFN 1280->5120->1280 at M = 1, 32, 1500, run (i) on
one core and run (ii) on every core of this process, CPU model printed; the
clip's Q4 GEMM time is extrapolated from those x layer counts.  Emitted by
rank 0 at every world size.  Multi-rank runs use a gloo (host) group for the
barriers and the MAX of the timed seconds: RCCL is never initialised.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "whisper-burn_amd"))

METRIC = "real-time factor (audio-s/wall-s) Whisper Large-V3 Q4 @1/2/4/8 MI355X"
CLIP_SECONDS = 30.0
PEAK_MFMA_TFLOPS = 2500.0  # dense f16/bf16, MI355X_MICROARCH.md:43
PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md:36


def clip_q4_gflop(cfg: dict, tokens: float) -> float:
    """Algorithmic Q4 GEMM GFLOP per clip."""
    D, T = cfg["n_audio_state"], cfg["n_audio_ctx"]
    Dt = cfg["n_text_state"]
    enc = cfg["n_audio_layer"] * 2 * T * (4 * D * D + 2 * 4 * D * D)
    cross = cfg["n_text_layer"] * 2 * T * 2 * Dt * D
    per_tok = cfg["n_text_layer"] * 2 * (6 * Dt * Dt + 2 * 4 * Dt * Dt)
    return (enc + cross + per_tok * (4 + tokens)) * 1e-9


def clip_ids(rank: int, B: int, warmup: int, steps: int) -> list[list[int]]:
    """Global clip index of every clip a rank runs, per step (warmup first).
    Ranks own disjoint contiguous ranges: independent clips, no exchange."""
    per_rank = (warmup + steps) * B
    return [[rank * per_rank + s * B + i for i in range(B)] for s in range(warmup + steps)]


def max_over_ranks(x: float, dist, device) -> float:
    """The job's wall time: max of the ranks' timed-region seconds (the only
    collective in the run; not on the data path)."""
    if dist is None:
        return x
    import torch

    t = torch.tensor([x], device=device, dtype=torch.float64)  # device "cpu": gloo
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def init_dist():
    """Process group of a multi-rank run: gloo over the host.  The only
    cross-rank traffic is the barriers and one MAX of the timed-region seconds,
    so RCCL is never initialised (no collective on the data
    path).  Rendezvous from the torch.distributed.run environment."""
    import torch.distributed as dist

    dist.init_process_group("gloo")
    return dist


def baseline_config_label(variant: str, weights: str, precision: str, clips: int) -> str:
    """Which BASELINE.json configuration this run is (configs 2-5), or why
    it is none."""
    if precision != "f16x2":
        return "not a BASELINE config: f16 operands (--precision f16)"
    if variant == "medium" and weights == "q4_0":
        return "BASELINE config 2" + ("" if clips == 1 else f" at {clips} clips (config 2 is one clip)")
    if variant == "large_v3" and weights == "f16":
        return f"BASELINE config 5 (f16 weights), {clips} clip{'s' if clips != 1 else ''} per GPU"
    if variant == "large_v3" and weights == "q4_0":
        if clips == 1:
            return "BASELINE config 3 (batch 1)"
        if clips == 32:
            return "BASELINE config 4 shard (32 of its 256 clips per GPU)"
        return f"Large-V3 Q4_0 at {clips} clips per GPU (between BASELINE configs 3 and 4)"
    return f"not a BASELINE config: {variant} {weights}"


def job_rtf(world: int, B: int, steps: int, elapsed: float) -> float:
    """Whole-job real-time factor: audio seconds of all ranks' clips / wall s."""
    return world * B * steps * CLIP_SECONDS / elapsed


def _pmc_kernels(workload: dict):
    """Kernel table of the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, written by scripts/pmc_summary.py from separate
    FETCH_SIZE / WRITE_SIZE passes, FETCH_SIZE doubled per MI355X_MICROARCH.md
    'HBM'), or None when absent or when it profiled another workload (variant,
    weights, precision, clips): a summary is never borrowed across runs."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("workload") != workload:
        return None
    return d.get("kernels", {})


def pmc_traffic(kernel: str, workload: dict):
    """HBM bytes per launch of `kernel` (all its launches), or None."""
    k = _pmc_kernels(workload)
    v = None if k is None else k.get(kernel)
    return None if v is None else v.get("hbm_bytes_per_launch")


def pmc_traffic_grid(kernel: str, grid_items: int, workload: dict):
    """HBM bytes per launch of `kernel` at one dispatch size (total
    work-items), or None."""
    k = _pmc_kernels(workload)
    try:
        return k[kernel]["by_grid_items"][str(grid_items)]["hbm_bytes_per_launch"]
    except (TypeError, KeyError):
        return None


def pmc_traffic_xattn_probe(rows: int, heads: int, d_model: int, workload: dict):
    """HBM bytes of one decode-step cross-attention at the bench probe's shape
    (all `rows` clips in one launch), each kernel looked up at its own grid
    (work-items): xattn_q (H x D/64 x ceil(rows/32) workgroups of 128),
    xattn_main (8 frame splits x 512 work-items per row), xattn_out (512
    work-items per head per 4 rows) -- the launches `achieved` is timed over.
    None if not measured for this workload."""
    parts = [pmc_traffic_grid("xattn_q_kernel", heads * (d_model // 64) * ((rows + 31) // 32) * 128, workload),
             pmc_traffic_grid("xattn_main_kernel", 8 * 512 * rows, workload),
             pmc_traffic_grid("xattn_out_kernel", heads * 512 * ((rows + 3) // 4), workload)]
    return None if any(p is None for p in parts) else sum(parts)


def in_graph_xattn(rows: int, heads: int, d_model: int, workload: dict):
    """Sum of the in-graph average durations (us) of xattn_q, xattn_main and
    xattn_out at the decode group's grids, from the committed chain trace
    (profiles/xattn_in_graph.json) of this workload, or None."""
    try:
        with open(os.path.join(REPO, "profiles", "xattn_in_graph.json")) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("workload") != workload:
        return None
    # grids in work-items: xattn_q (H, D/64, ceil(rows/32)) x 128 threads,
    # xattn_main (8 splits, rows) x 512, xattn_out (H, ceil(rows/4)) x 512
    want = {"xattn_q_mfma_kernel": [heads * 128, d_model // 64, (rows + 31) // 32],
            "xattn_main_kernel": [4096, rows, 1], "xattn_out_kernel": [heads * 512, (rows + 3) // 4, 1]}
    tot = 0.0
    for k, grid in want.items():
        hit = [e for e in d.get("kernels", []) if e["kernel"] == k and list(e["grid"]) == grid]
        if not hit:
            return None
        tot += hit[0]["avg_us"]
    return tot


def decode_overlap(workload: dict):
    """The committed wall-time view of the decode (profiles/decode_overlap.json,
    scripts/decode_overlap.py over the rocprofv3 kernel trace of this
    workload), or None."""
    try:
        with open(os.path.join(REPO, "profiles", "decode_overlap.json")) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    return d if d.get("workload") == workload else None


def decode_step_bytes(cfg: dict, B: int, groups: int, kv_cache: bool, weights: str, ns: int, kv_avg: float) -> dict:
    """Algorithmic HBM bytes of one greedy decode step over B clips in `groups`
    decode groups (each group replays its own step graph, so it streams the
    weights and the logits table itself), SURVEY §8(d):
      cross-attention state: every clip's encoder output as f16 planes
        (ns halves per element) + raw Wk, Wv per group -- or, for few-clip
        groups, the reference's cached K and V (f32) -- per layer;
      decoder Q4 weights (qkv, out, cq, cout, fc1, fc2: 14 D^2) per group;
      self-attention KV cache, K and V f32, kv_avg entries per clip and layer;
      the tied-embedding logits table (f16 pairs) per group."""
    D, T, L, V = cfg["n_text_state"], cfg["n_audio_ctx"], cfg["n_text_layer"], cfg["n_vocab"]
    wb = 2.0 if weights == "f16" else 18.0 / 32.0
    xattn = B * T * D * 4.0 * 2 if kv_cache else B * T * D * 2.0 * ns + groups * 2 * D * D * wb
    w = groups * 14 * D * D * wb
    self_kv = B * kv_avg * D * 4.0 * 2
    logits = groups * ((V + 127) // 128 * 128) * D * 2.0 * ns
    per = {"cross_attention": L * xattn, "weights": L * w, "self_kv": L * self_kv, "logits_table": logits}
    per["total"] = sum(per.values())
    return per


def cpu_threads() -> int:
    """Host cores this process may use: the affinity mask, capped by
    OMP_NUM_THREADS where the box sets it (the GPU box's CPU share)."""
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


CPU_ROWS = (1, 32, 1500)


def cpu_shape_times(D: int, nthreads: int, sample_rows: int) -> dict:
    """Q4Linear D x D and Q4FFN D -> 4D -> D on the reference's
    CPU path (dequantize + naive i-j-l matmul, tests.rs:60-87,172-184), at
    M = 1, 32, 1500 rows.  The naive loop is linear in M, so M = 1500 is timed
    on min(sample_rows, 1500) rows and scaled by 1500 / rows (the per-call
    dequant, < 2 % of such a call, is scaled with it).  Returns {name: {"rows_timed", "s", "gflops"}}."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np

    import oracle

    rng = np.random.default_rng(0)
    F = 4 * D
    w = {n: oracle.quantize_convert_np((rng.standard_normal(a * b) * 0.02).astype(np.float32))
         for n, a, b in (("lin", D, D), ("fc1", F, D), ("fc2", D, F))}
    b_d = (rng.standard_normal(D) * 0.01).astype(np.float32)
    b_f = (rng.standard_normal(F) * 0.01).astype(np.float32)
    out = {}
    for m in CPU_ROWS:
        r = min(m, sample_rows)
        x = rng.standard_normal(r * D).astype(np.float32)
        for name, flop_per_row in (("q4linear", 2.0 * D * D), ("q4ffn", 4.0 * D * F)):
            t0 = time.perf_counter()
            if name == "q4linear":
                oracle.cpu_linear(w["lin"], b_d, x, r, D, D, nthreads)
            else:
                oracle.cpu_ffn(w["fc1"], b_f, w["fc2"], b_d, x, r, D, F, nthreads)
            t = time.perf_counter() - t0
            s = t * m / r
            out[f"{name}_M{m}"] = {"rows_timed": r, "s": round(s, 5), "gflops": round(flop_per_row * m / s * 1e-9, 3)}
    return out


def cpu_clip_seconds(cfg: dict, shapes: dict, tokens: float) -> float:
    """Extrapolated CPU seconds of one clip's Q4 GEMMs: encoder
    and cross-K/V projections at M = 1500 rows, prompt + greedy decode at
    M = 1 row per token (the reference decodes one clip at a time), from the
    per-shape timings x layer counts.  The model's other ops are not counted:
    a lower bound on the reference CPU path's clip time."""
    lin = lambda m: shapes[f"q4linear_M{m}"]["s"]
    ffn = lambda m: shapes[f"q4ffn_M{m}"]["s"]
    enc = cfg["n_audio_layer"] * (4 * lin(1500) + ffn(1500))
    cross = cfg["n_text_layer"] * 2 * lin(1500)
    per_tok = cfg["n_text_layer"] * (6 * lin(1) + ffn(1))
    return enc + cross + per_tok * (4 + tokens)


def cpu_baseline(cfg: dict, rows: int, tokens: float) -> dict:
    """The reference's CPU dequant -> GEMM path timed on this box:
    run (i) one core, as the reference runs it; run (ii) all cores of this
    process (OpenMP over outputs, this build's parallelisation).  value = run
    (i)'s extrapolated real-time factor of one clip's Q4 GEMMs."""
    D = cfg["n_audio_state"]
    n_all = cpu_threads()
    t0 = time.perf_counter()
    single = cpu_shape_times(D, 1, rows)
    multi = cpu_shape_times(D, n_all, 1500) if n_all > 1 else single
    wall = time.perf_counter() - t0
    c1 = cpu_clip_seconds(cfg, single, tokens)
    cn = cpu_clip_seconds(cfg, multi, tokens)
    return {"value": round(CLIP_SECONDS / c1, 4), "unit": "audio-s/wall-s", "cores": 1, "kind": "port",
            "cpu_model": cpu_model(),
            "sample": f"Q4Linear {D}x{D} and Q4FFN {D}->{4 * D}->{D} at M = 1, 32, 1500 rows on the reference's CPU "
                      f"path (dequantize + naive f32 matmul, tests.rs:60-87,172-184, oracle/q4_oracle.c); run (i) 1 "
                      f"core (M = 1500 timed on {min(rows, 1500)} rows, scaled), run (ii) {n_all} cores (OpenMP over "
                      f"outputs, all 1500 rows); value = 30 s / one clip's Q4 GEMM seconds extrapolated from the "
                      f"shape timings x layer counts ({tokens:.0f} tokens, M = 1 decode); {wall:.1f} s of CPU timing",
            "single_core": {"cores": 1, "clip_q4_s_extrapolated": round(c1, 2), "shapes": single},
            "all_cores": {"cores": n_all, "value": round(CLIP_SECONDS / cn, 4),
                          "clip_q4_s_extrapolated": round(cn, 2), "shapes": multi}}


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv: list[str]) -> int:
    """`--gpus N` (N > 1) started without a torch.distributed.run environment:
    start N rank processes of this script (RANK / WORLD_SIZE / LOCAL_RANK /
    MASTER_ADDR=127.0.0.1 / MASTER_PORT set), one per GPU, and wait for them.
    This parent never initialises HIP (it imports neither torch nor the
    product libraries), so no process that touched the GPU is replaced or
    forks.  If a rank fails, the others are stopped (their exact PIDs) and the
    failing rank's exit status is returned."""
    import subprocess

    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    pending = set(range(n))
    while pending:
        for i in sorted(pending):
            c = procs[i].poll()
            if c is None:
                continue
            pending.discard(i)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                print(f"bench.py: rank {i} exited with status {c}; stopping the other ranks", file=sys.stderr,
                      flush=True)
                for j in pending:
                    procs[j].terminate()
        time.sleep(0.1)
    return rc


def dry_run(args, rank: int, world: int) -> None:
    """`--dry-run`: the launch, rendezvous, barrier and max-over-ranks logic of
    a multi-rank run with no GPU work (the CPU test of `--gpus N`).  Each rank
    'runs' its clip shard (clip_ids) for a rank-dependent time; rank 0 prints
    the one JSON line with n_gpus = world.

    Test-only fault injection: BENCH_DRY_RUN_FAIL="rank:status" makes that
    rank print its PID and exit with `status` before the rendezvous, so the
    other ranks block in it until launch_ranks stops them
    (tests/test_bench_dist.py::test_bench_gpus_rank_failure_stops_the_others)."""
    print(f"bench.py: rank {rank} pid {os.getpid()}", file=sys.stderr, flush=True)
    fail = os.environ.get("BENCH_DRY_RUN_FAIL", "")
    if fail:
        fr, status = (int(v) for v in fail.split(":"))
        if fr == rank:
            sys.exit(status)
    dist = init_dist() if world > 1 else None
    ranks_seen = 1
    if dist is not None:
        import torch

        t = torch.ones(1, dtype=torch.float64)
        dist.all_reduce(t)
        ranks_seen = int(t.item())
        dist.barrier()
    t0 = time.perf_counter()
    ids = clip_ids(rank, args.clips_per_gpu, args.warmup, args.steps)
    time.sleep(0.01 * (1 + rank))
    elapsed = max_over_ranks(time.perf_counter() - t0, dist, "cpu")
    if rank == 0:
        assert world == args.gpus, f"world size {world} != --gpus {args.gpus}"
        line = {"metric": METRIC, "value": round(job_rtf(world, args.clips_per_gpu, args.steps, elapsed), 3),
                "unit": "audio-s/wall-s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(elapsed / args.steps * 1e3, 3), "dry_run": True,
                "backend": None if dist is None else dist.get_backend(), "ranks_seen": ranks_seen,
                "clips_rank0": sum(len(s) for s in ids)}
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); > 1 without a torch.distributed.run environment starts them itself")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--variant", default="large_v3", choices=["large_v3", "medium", "tiny_test"])
    ap.add_argument("--clips-per-gpu", type=int, default=32)
    ap.add_argument("--max-tokens", type=int, default=224)
    ap.add_argument("--lang", type=int, default=50259, help="language token; -1 = auto-detect")
    ap.add_argument("--precision", default="f16x2", choices=["f16x2", "f16"])
    ap.add_argument("--weights", default="q4_0", choices=["q4_0", "f16"],
                    help="linear weights: Q4_0 (default) or unquantized f16 (BASELINE config 5)")
    ap.add_argument("--audio", action="store_true",
                    help="start from 16 kHz samples in HBM: the GPU log-mel front-end (wa_log_mel) runs inside "
                         "the timed region")
    ap.add_argument("--fixed-length", action="store_true", help="ignore EOT (always max-tokens steps)")
    ap.add_argument("--sequential", action="store_true",
                    help="one wa_transcribe per step (no encoder / decode pipelining across steps)")
    ap.add_argument("--seq-steps", type=int, default=3,
                    help="pipelined runs: batches then timed one wa_transcribe each, for value_sequential "
                         "(0 = skip)")
    ap.add_argument("--cpu-rows", type=int, default=160,
                    help="rows the single-core CPU baseline times at M = 1500 (scaled to 1500)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--dry-run", action="store_true",
                    help="launch / rendezvous / max-over-ranks only, no GPU work (CPU test of --gpus N)")
    args = ap.parse_args()

    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr, flush=True)
        sys.exit(2)
    if args.dry_run:
        dry_run(args, rank, world)
        return
    import numpy as np
    import torch

    import whisper_amd
    import wq4

    n_dev = wq4.device_count()
    if n_dev < world:
        print(f"bench.py: --gpus {world} but {n_dev} HIP device(s) visible", file=sys.stderr, flush=True)
        sys.exit(2)
    torch.cuda.set_device(local_rank)
    dist = init_dist() if world > 1 else None
    prec = wq4.PREC_F16X2 if args.precision == "f16x2" else wq4.PREC_F16
    t_load = time.perf_counter()
    model = whisper_amd.WhisperModel(args.variant, args.seed, max_batch=args.clips_per_gpu, device=local_rank,
                                     precision=prec, weights=args.weights)
    t_load = time.perf_counter() - t_load
    cfg = model.config
    B = args.clips_per_gpu
    n_mels = cfg["n_mels"]

    def batch(ids: list[int]):
        arr = np.stack([whisper_amd.synth_uniform(0x5EED0000 + c, "mel", n_mels * 3000, -1.5, 1.0) for c in ids])
        return torch.from_numpy(arr.reshape(len(ids), n_mels, 3000)).to(f"cuda:{local_rank}")

    def audio_batch(ids: list[int]):
        # speech-like synthetic audio: two per-clip tones under a 4 Hz envelope + noise, [B, 480000] f32
        t = np.arange(480000, dtype=np.float64) / 16000.0
        rows = []
        for c in ids:
            rng = np.random.default_rng(0x5EED0000 + c)
            f1, f2 = 100.0 + 3.0 * (c % 97), 900.0 + 17.0 * (c % 89)
            x = 0.3 * (0.5 + 0.5 * np.sin(2 * np.pi * 4.0 * t + c)) * np.sin(2 * np.pi * f1 * t)
            x += 0.1 * np.sin(2 * np.pi * f2 * t) + 0.02 * rng.standard_normal(t.size)
            rows.append(x.astype(np.float32))
        return torch.from_numpy(np.stack(rows)).to(f"cuda:{local_rank}")

    make = audio_batch if args.audio else batch
    inputs = [make(ids) for ids in clip_ids(rank, B, args.warmup, args.steps)]  # resident in HBM before timing
    mel_buf = torch.empty((B, n_mels, 3000), device=f"cuda:{local_rank}", dtype=torch.float32)
    mel_ms = []

    def run(x):
        if not args.audio:
            return model.transcribe(x, lang, args.max_tokens, eot_stop=not args.fixed_length)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        whisper_amd.log_mel(x, n_mels, out=mel_buf)
        e1.record()
        toks = model.transcribe(mel_buf, lang, args.max_tokens, eot_stop=not args.fixed_length)
        mel_ms.append(e0.elapsed_time(e1))
        return toks

    lang = None if args.lang < 0 else args.lang
    # Pipelined (default for mel input): the timed steps are ONE
    # wa_transcribe_batches call over the K batches -- each next batch's conv
    # stem and first encoder layers run on a CU-masked stream beside the
    # current batch's decode (serving throughput); every batch's encoder and
    # decode run inside the timed region.  --sequential: one wa_transcribe per step.
    pipelined = not args.audio and not args.sequential
    eot = not args.fixed_length
    if pipelined:
        if args.warmup > 0:  # graphs, the masked stream and the overlap depth (a 1-step warmup runs 2 batches)
            warm = torch.stack(inputs[: args.warmup] if args.warmup >= 2 else [inputs[0], inputs[0]])
            model.transcribe_batches(warm, lang, args.max_tokens, eot_stop=eot)
            del warm
        timed_in = torch.stack(inputs[args.warmup:])
    else:
        for s in range(args.warmup):
            run(inputs[s])
    mel_ms.clear()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    model.profile_read(reset=True)
    model.profile_enable(True)
    ntok = []
    timings = []
    pipe = None
    t0 = time.perf_counter()
    if pipelined:
        for toks in model.transcribe_batches(timed_in, lang, args.max_tokens, eot_stop=eot):
            ntok += [len(t) for t in toks]
        timings = [model.last_timings()]
        pipe = model.pipeline_stats()
    else:
        for s in range(args.steps):
            toks = run(inputs[args.warmup + s])
            ntok += [len(t) for t in toks]
            timings.append(model.last_timings())
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    model.profile_enable(False)
    prof = model.profile_read(reset=True)
    # The same batches one wa_transcribe each (the reference's loop: one
    # transcribe, encoder then decode, per call) -- reported beside the
    # pipelined `value`, never as it.
    seq_elapsed = None
    n_seq = min(args.seq_steps, args.steps) if pipelined else 0
    if n_seq > 0:
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        t2 = time.perf_counter()
        for s in range(n_seq):
            model.transcribe(inputs[args.warmup + s], lang, args.max_tokens, eot_stop=eot)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        seq_elapsed = max_over_ranks(time.perf_counter() - t2, dist, "cpu")
    # PCIe-inclusive figure (never `value`): one batch's inputs from pinned host
    # memory to HBM, timed after the timed steps and added per step
    host_in = inputs[0].cpu().pin_memory()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(3):
        inputs[0].copy_(host_in, non_blocking=True)
    torch.cuda.synchronize()
    h2d_s = (time.perf_counter() - t1) / 3
    elapsed_pcie = max_over_ranks(elapsed + args.steps * h2d_s, dist, "cpu")
    elapsed = max_over_ranks(elapsed, dist, "cpu")
    clips = world * B * args.steps
    value = job_rtf(world, B, args.steps, elapsed)

    group_rows = whisper_amd.decode_group_rows(B)
    probe = model.probe_kernels(group_rows, iters=20) if rank == 0 else None
    if rank == 0:
        workload = {"variant": args.variant, "weights": args.weights, "precision": args.precision, "clips": B}
        q4 = prof["q4_gemm"]
        mean_tok = float(np.mean(ntok)) if ntok else 0.0
        steps_run = float(np.mean([t["steps"] for t in timings])) if timings else 0.0
        # north-star kernel: the encoder's Q4 MFMA GEMMs, timed live per launch;
        # the kernel that ran them at this row count (tile or ring kernel)
        enc_rows = B * cfg["n_audio_ctx"]
        enc_kernel = wq4.gemm_kernel_name(cfg["n_audio_state"], cfg["n_audio_state"], enc_rows)
        q4_tf = q4["gflop"] / (q4["ms"] * 1e-3) * 1e-3 if q4["ms"] > 0 else 0.0
        roof_q4 = {"bound": "mfma", "achieved": round(q4_tf, 2), "peak": PEAK_MFMA_TFLOPS, "unit": "TFLOP/s",
                   "frac": round(q4_tf / PEAK_MFMA_TFLOPS, 4),
                   "traffic": pmc_traffic(enc_kernel, workload),
                   "kernel": f"{enc_kernel} (encoder Q4 GEMMs, M = {enc_rows})",
                   "launches": q4["launches"], "avg_us": round(q4["ms"] / max(1, q4["launches"]) * 1e3, 2),
                   "gpu_ms_per_step": round(q4["ms"] / args.steps, 2)}
        # decode phase: cross-attention (HBM stream of the encoder-output planes), probed after the timed steps
        xa = probe["cross_attention"]
        xa_gbs = xa["bytes"] / (xa["us"] * 1e-6) * 1e-9
        groups = -(-B // group_rows)
        kv = xa["kv_cache"]  # few clips: the GEMV over the cached cross K / V (one launch)
        ig = None if kv else in_graph_xattn(group_rows, cfg["n_text_head"], cfg["n_text_state"], workload)
        xa_kernel = ("cross-attention over the cached cross K / V: cross_attn_kv_kernel" if kv else
                     "cross-attention over the encoder output: xattn_q + xattn_main + xattn_out")
        roof_xa = {"bound": "hbm", "achieved": round(xa_gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                   "frac": round(xa_gbs / PEAK_HBM_GBS, 4),
                   "traffic": None if kv else pmc_traffic_xattn_probe(group_rows, cfg["n_text_head"],
                                                                      cfg["n_text_state"], workload),
                   "kernel": f"{xa_kernel} "
                             f"(decode step, Tq = 1, {group_rows} clips per launch = one of {groups} decode groups)",
                   "avg_us": round(xa["us"], 2), "bytes_per_launch": xa["bytes"],
                   "in_graph_avg_us": None if ig is None else round(ig, 2),
                   "in_graph_frac": None if ig is None else round(xa["bytes"] / (ig * 1e-6) * 1e-9 / PEAK_HBM_GBS, 4),
                   # summed over both decode groups' launches (they overlap in wall time)
                   "gpu_ms_per_step": round(xa["us"] * 1e-3 * cfg["n_text_layer"] * steps_run * groups, 2)}
        dq = probe["decode_fc1"]
        roof_dq = {"bound": "hbm", "achieved": round(dq["bytes"] / (dq["us"] * 1e-6) * 1e-9, 1),
                   "peak": PEAK_HBM_GBS, "unit": "GB/s",
                   "frac": round(dq["bytes"] / (dq["us"] * 1e-6) * 1e-9 / PEAK_HBM_GBS, 4), "traffic": None,
                   "kernel": f"q4_gemm_decode_kernel (decode-step fc1, split-K, {group_rows} rows)",
                   "avg_us": round(dq["us"], 2),
                   "tflops": round(dq["flops"] / (dq["us"] * 1e-6) * 1e-12, 2)}
        # the decode step as a whole: algorithmic bytes per step / measured wall time per step
        phase = {k: float(np.mean([t[k] for t in timings])) for k in ("encoder_ms", "cross_kv_ms", "prompt_ms",
                                                                         "decode_ms")}
        ns = 2 if prec == wq4.PREC_F16X2 else 1
        kv_avg = 4.0 + (steps_run + 1) / 2.0  # prompt (4) + the steps so far, averaged over the loop
        sb = decode_step_bytes(cfg, B, groups, kv, args.weights, ns, kv_avg)
        step_ms = phase["decode_ms"] / max(1.0, steps_run)
        ds_gbs = sb["total"] / (step_ms * 1e-3) * 1e-9
        roof_ds = {"bound": "hbm", "achieved": round(ds_gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                   "frac": round(ds_gbs / PEAK_HBM_GBS, 4), "traffic": None,
                   "kernel": f"one greedy decode step (all {groups} decode groups, {B} clips), wall time",
                   "ms_per_step": round(step_ms, 4), "bytes_per_step": {k: int(v) for k, v in sb.items()},
                   "kv_avg": kv_avg, "floor_ms_per_step": round(sb["total"] / (PEAK_HBM_GBS * 1e9) * 1e3, 4)}
        # wall-time share (like for like with the serial encoder GEMMs): the
        # groups' launches overlap, so summed GPU time is scaled by the
        # union / sum of the same family's intervals in the committed trace
        ov = decode_overlap(workload)
        fam = None if ov is None else ov["families"].get("cross_attention")
        if fam is not None:
            roof_xa["wall_ms_per_step"] = round(roof_xa["gpu_ms_per_step"] * fam["union_over_sum"], 2)
            roof_xa["wall_ms_source"] = "profiles/decode_overlap.json (union / sum of the family's in-graph intervals)"
        else:  # no committed trace of this workload: the groups' launches taken as perfectly overlapped
            roof_xa["wall_ms_per_step"] = round(roof_xa["gpu_ms_per_step"] / groups, 2)
            roof_xa["wall_ms_source"] = f"estimate: summed GPU ms / {groups} decode groups (no committed trace)"
        main = None if ov is None else ov["families"].get("xattn_main_kernel")
        if main and not kv:
            mb = group_rows * cfg["n_audio_ctx"] * cfg["n_text_state"] * 2.0 * ns  # planes per launch
            cg = mb * main["launches"] / (main["union_us"] * 1e-6) * 1e-9
            roof_xa["concurrent_main"] = {
                "source": "profiles/decode_overlap.json", "launches": main["launches"],
                "sum_us": main["sum_us"], "union_us": main["union_us"], "achieved_gbs": round(cg, 1),
                "frac": round(cg / PEAK_HBM_GBS, 4),
                "note": "encoder-plane bytes of every xattn_main launch of both groups over the union of their "
                        "intervals (wall time with at least one running)"}
        xa_wall = roof_xa["wall_ms_per_step"]
        roof_q4["wall_ms_per_step"] = roof_q4["gpu_ms_per_step"]  # one stream: GPU time is wall time
        dominant = roof_xa if xa_wall > roof_q4["wall_ms_per_step"] else roof_q4
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "audio-s/wall-s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "fp16x2" if prec == wq4.PREC_F16X2 else "fp16", "data": "synthetic",
            "config": {"workload": f"Whisper {args.variant} {args.weights.upper()}, {B} synthetic 30-s clips per GPU per step "
                                   f"({baseline_config_label(args.variant, args.weights, args.precision, B)})"
                                   f"{', from audio' if args.audio else ''}, greedy KV-cached decode, max {args.max_tokens} "
                                   f"tokens, {'fixed length' if args.fixed_length else 'EOT stop'}",
                       "model": f"whisper-{args.variant.replace('_', '-')}-{args.weights} (synthetic weights)",
                       "global_batch": clips // args.steps, "seq_len": cfg["n_audio_ctx"],
                       "parallelism": f"replicas{world} (independent clips, no collectives)"},
            "roofline": dominant,
            "roofline_q4_gemm": roof_q4,
            "roofline_cross_attention": roof_xa,
            "roofline_decode_gemm": roof_dq,
            "roofline_decode_step": roof_ds,
            "kernels": {k: {"launches": v["launches"], "ms": round(v["ms"], 3),
                            "tflops": round(v["gflop"] / (v["ms"] * 1e-3) * 1e-3, 2) if v["ms"] else None,
                            "gbs": round(v["gb"] / (v["ms"] * 1e-3), 1) if v["ms"] else None}
                        for k, v in prof.items()},
            "tokens_per_clip": round(mean_tok, 2),
            "phase_ms": {k: round(v, 3) for k, v in phase.items()},
            "decode_steps": [t["steps"] for t in timings],
            "pipeline": None if pipe is None else dict(pipe, note=(
                "one wa_transcribe_batches call over the timed steps: each next batch's conv stem + first "
                "overlap_layers encoder layers on a CU-masked stream beside the current decode; phase_ms.encoder_ms "
                "= encoder time per batch not hidden by a decode; the Q4 GEMM events cover the full-width "
                "launches only")),
            "input": "16 kHz audio in HBM (GPU log-mel timed)" if args.audio else "log-mel in HBM",
            "input_h2d_ms_per_step": round(h2d_s * 1e3, 3),
            "value_pcie_inclusive": round(job_rtf(world, B, args.steps, elapsed_pcie), 3),
            "value_sequential": None if seq_elapsed is None else round(job_rtf(world, B, n_seq, seq_elapsed), 3),
            "ms_per_step_sequential": None if seq_elapsed is None else round(seq_elapsed / n_seq * 1e3, 3),
            "value_note": ("value: pipelined serving throughput (one wa_transcribe_batches call; the next batch's "
                           "encoder beside the current decode); value_sequential: the same batches one "
                           "wa_transcribe each, the reference's transcribe-per-call loop (whisper.rs:51-128) -- "
                           "the like-for-like figure for the reference (BASELINE.md section 3); both with the "
                           "mels resident in HBM, value_pcie_inclusive adds their H2D copy")
            if pipelined else "one wa_transcribe per step (the reference's loop), mels resident in HBM",
            "log_mel_ms": round(float(np.mean(mel_ms)), 3) if mel_ms else None,
            "model_load_s": round(t_load, 2),
        }
        line["cpu_baseline"] = None if args.no_cpu_baseline else cpu_baseline(model.config, args.cpu_rows, mean_tok)
        s = json.dumps(line)
        print(s, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(s + "\n")
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
