"""Q4 GEMM microbenchmark: kernel time per Whisper shape, HIP-event timed.

    python whisper-burn_amd/tools/q4_bench.py [--json out.json] [--iters 20]

Times wq4_linear_forward_tiled (the GEMM alone, activations already in the
A-tiled operand layout, as the model path feeds it), captured `iters` times
into one HIP graph on a side stream so small-M launches are not hidden by
Python call overhead (--no-graph: plain back-to-back launches), and reports TFLOP/s and algorithmic GB/s against the MI355X peaks
(2.5 PF dense f16/bf16 MFMA, 8.0 TB/s HBM; MI355X_MICROARCH.md:36,43).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle"))
import wq4  # noqa: E402

PEAK_TFLOPS = 2500.0
PEAK_GBS = 8000.0


def rand_q4(n: int, k: int, seed: int) -> np.ndarray:
    """Random Q4_0 bytes (valid nibbles, f16 scales ~ 0.02/7) -- fast, no oracle."""
    rng = np.random.default_rng(seed)
    nb = n * k // 32
    blk = np.empty((nb, 18), np.uint8)
    d = (rng.uniform(0.5, 1.5, nb) * 0.02 / 7).astype(np.float16)
    blk[:, :2] = d.view(np.uint8).reshape(nb, 2)
    blk[:, 2:] = rng.integers(0, 256, (nb, 16), dtype=np.uint8)
    return blk.ravel()


def bench_shape(torch, m: int, n: int, k: int, prec: int, policy: int, iters: int, warmup: int = 3,
                graph: bool = True, cold: int = 0) -> dict:
    """cold > 0: the graph cycles through `cold` distinct weight tensors (more
    bytes than the caches hold), so every launch reads its weights from HBM,
    as the decoder's layer-by-layer chain does."""
    L = wq4.lib()
    t = wq4.Q4Tensor.from_q4_bytes(rand_q4(n, k, n * 31 + k), [n, k])
    ts = [t] + [wq4.Q4Tensor.from_q4_bytes(rand_q4(n, k, n * 31 + k + i), [n, k]) for i in range(1, cold)]
    it = [0]
    x = torch.randn((m, k), device="cuda:0", dtype=torch.float32)
    atb = L.wq4_atiled_bytes(m, k, prec)
    at = torch.empty(atb, dtype=torch.uint8, device="cuda:0")
    y = torch.empty((m, n), device="cuda:0", dtype=torch.float32)
    side = torch.cuda.Stream()
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        st = ctypes.c_void_p(side.cuda_stream)
        wq4.check(L.wq4_tile_activations(ctypes.c_void_p(x.data_ptr()), m, k, k, prec,
                                         ctypes.c_void_p(at.data_ptr()), atb, st))
        wq4.set_kernel_policy(policy)

        def run():
            w = ts[it[0] % len(ts)]
            it[0] += 1
            wq4.check(L.wq4_linear_forward_tiled(w.handle, None, ctypes.c_void_p(at.data_ptr()), None,
                                                 ctypes.c_void_p(y.data_ptr()), m, 0, prec, st))

        for _ in range(warmup):
            run()
        side.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if graph:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=side):
                for _ in range(iters):
                    run()
            g.replay()
            side.synchronize()
            e0.record(side)
            g.replay()
            e1.record(side)
        else:
            e0.record(side)
            for _ in range(iters):
                run()
            e1.record(side)
        side.synchronize()
    ms = e0.elapsed_time(e1) / iters
    wq4.set_kernel_policy(0)
    flops = 2.0 * m * n * k
    bytes_ = n * k * 18 / 32 + m * k * 4 + m * n * 4
    return {"m": m, "n": n, "k": k, "prec": "f16x2" if prec == 0 else "f16",
            "kernel": {0: "auto", 1: "prefill", 2: "decode"}[policy], "us": ms * 1e3,
            "tflops": flops / (ms * 1e-3) / 1e12, "frac_mfma": flops / (ms * 1e-3) / 1e12 / PEAK_TFLOPS,
            "gbs": bytes_ / (ms * 1e-3) / 1e9, "frac_hbm": bytes_ / (ms * 1e-3) / 1e9 / PEAK_GBS}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--decode-only", action="store_true")
    ap.add_argument("--shape", default=None, help="m,n,k: one prefill-kernel shape only (profiling)")
    ap.add_argument("--prec", type=int, default=0, help="with --shape: 0 f16x2, 1 f16")
    ap.add_argument("--cold", type=int, default=0, help="decode shapes: cycle through N weight tensors")
    args = ap.parse_args()
    import torch

    rows = []
    if args.shape:
        m, n, k = (int(v) for v in args.shape.split(","))
        rows.append(bench_shape(torch, m, n, k, args.prec, 1, args.iters, graph=not args.no_graph))
        args.decode_only = True
        enc_m = []
    enc_m = [1500, 48000] if not args.quick else [1500, 12000]
    for prec in (() if args.shape else (wq4.PREC_F16X2, wq4.PREC_F16)):
        for (n, k) in [(1280, 1280), (3840, 1280), (5120, 1280), (1280, 5120)]:
            for m in ([] if args.decode_only else enc_m):
                rows.append(bench_shape(torch, m, n, k, prec, 1, args.iters, graph=not args.no_graph))
            for m in (1, 16, 32, 64):
                rows.append(bench_shape(torch, m, n, k, prec, 2, args.iters, graph=not args.no_graph,
                                        cold=args.cold))
    for r in rows:
        print(f"{r['kernel']:8s} {r['prec']:6s} M={r['m']:6d} N={r['n']:5d} K={r['k']:5d}  {r['us']:9.1f} us  "
              f"{r['tflops']:7.1f} TF/s ({100 * r['frac_mfma']:5.1f}% MFMA)  {r['gbs']:7.0f} GB/s "
              f"({100 * r['frac_hbm']:5.1f}% HBM)", flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump({"rows": rows, "time": time.time()}, f, indent=1)


if __name__ == "__main__":
    main()
