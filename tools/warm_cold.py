"""How much of a decode-size Q4 GEMM is weight-fetch latency: the 8-wave
decode kernel (kernel 2) at ROWS rows, 200 launches captured in one HIP
graph (as in the decode step), cycling over NT distinct weight copies:
NT = 1 keeps the weights in L2, a few dozen copies spill L2 but stay in
the 256 MB MALL, enough copies to exceed the MALL read HBM.  Prints the
average per-launch time per (shape, NT).

    ROWS=16 python tools/warm_cold.py          (env: ROWS, LAUNCHES, VARIANTS_ONLY=1
                                                skips the copies sweep)
"""
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "whisper-burn_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))

import oracle  # noqa: E402
import wq4  # noqa: E402

ROWS = int(os.environ.get("ROWS", "16"))
LAUNCHES = int(os.environ.get("LAUNCHES", "200"))
CASES = [((1280, 1280), (1, 24, 400)), ((5120, 1280), (1, 8, 100))]


def main():
    L = wq4.lib()
    vp = ctypes.c_void_p
    s = torch.cuda.Stream()
    st = vp(s.cuda_stream)
    wq4.check(L.wq4_prepare_stream(0, st))
    # floor: a one-element fill (one tiny kernel) per launch in the same graph shape
    tiny = torch.zeros(1, device="cuda")
    with torch.cuda.stream(s):
        tiny.fill_(1.0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for i in range(LAUNCHES):
            tiny.fill_(float(i))
    times = []
    for _ in range(7):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(s):  # replay() launches on the current stream
            a.record(s)
            g.replay()
            b.record(s)
        torch.cuda.synchronize()
        times.append(a.elapsed_time(b) * 1e3 / LAUNCHES)
    print(f"one-element fill: median {np.median(times[1:]):6.2f} us/launch, min {min(times[1:]):6.2f}", flush=True)
    del g
    rng = np.random.default_rng(0)
    for (n, k), nts in ([] if os.environ.get("VARIANTS_ONLY") else CASES):
        q = oracle.quantize_convert_np((rng.standard_normal(n * k) * 0.05).astype(np.float32))
        x = torch.randn(ROWS, k, device="cuda")
        at = torch.empty(L.wq4_atiled_bytes(ROWS, k, 0), dtype=torch.uint8, device="cuda")
        wq4.check(L.wq4_tile_activations(vp(x.data_ptr()), ROWS, k, k, 0, vp(at.data_ptr()), at.numel(), st))
        y = torch.empty(ROWS, n, device="cuda")
        pool = [wq4.Q4Tensor.from_q4_bytes(q, [n, k], decode_step=False) for _ in range(max(nts))]
        torch.cuda.synchronize()
        for nt in nts:
            ws = pool[:nt]
            run = lambda t: wq4.check(L.wq4_gemm_tiled(t.handle, None, vp(at.data_ptr()), None, vp(y.data_ptr()),
                                                       None, ROWS, 0, 0, 2, st))
            with torch.cuda.stream(s):
                for t in ws:
                    run(t)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for i in range(LAUNCHES):
                    run(ws[i % nt])
            times = []
            for _ in range(7):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                with torch.cuda.stream(s):
                    a.record(s)
                    g.replay()
                    b.record(s)
                torch.cuda.synchronize()
                times.append(a.elapsed_time(b) * 1e3 / LAUNCHES)
            mb = n * k * 18 / 32 / 1e6
            print(f"N={n:5d} K={k:5d} rows={ROWS} copies={nt:4d} ({nt * mb:6.1f} MB): "
                  f"median {np.median(times[1:]):6.2f} us/launch, min {min(times[1:]):6.2f}", flush=True)
            del g
    # epilogue variants at one copy (L2-warm): what the decode step's
    # LayerNorm-fold producers / consumers add to the plain GEMM
    p = lambda t: None if t is None else vp(t.data_ptr())
    for n, k in ((1280, 1280), (5120, 1280), (1280, 5120)):
        q = oracle.quantize_convert_np((rng.standard_normal(n * k) * 0.05).astype(np.float32))
        t = wq4.Q4Tensor.from_q4_bytes(q, [n, k])
        x = torch.randn(ROWS, k, device="cuda")
        at = torch.empty(L.wq4_atiled_bytes(ROWS, k, 0), dtype=torch.uint8, device="cuda")
        wq4.check(L.wq4_tile_activations(vp(x.data_ptr()), ROWS, k, k, 0, vp(at.data_ptr()), at.numel(), st))
        y = torch.zeros(ROWS, n, device="cuda")
        yt = torch.zeros(L.wq4_atiled_bytes(ROWS, n, 0), dtype=torch.uint8, device="cuda")
        bias = torch.zeros(n, device="cuda")
        gam = torch.ones(n, device="cuda")
        stats_out = torch.zeros(ROWS * n // 16 * 2, device="cuda")
        stats_in = torch.zeros(ROWS * k // 16 * 2, device="cuda")
        stats_in[1::2] = 16.0
        wg = torch.zeros(n, device="cuda")
        prod = wq4.LnFold(gam.data_ptr(), yt.data_ptr(), stats_out.data_ptr(), None, None)
        cons = wq4.LnFold(None, None, None, stats_in.data_ptr(), wg.data_ptr())
        variants = {
            "plain": lambda: L.wq4_gemm_tiled(t.handle, p(bias), p(at), None, p(y), None, ROWS, 0, 0, 2, st),
            "residual": lambda: L.wq4_gemm_tiled(t.handle, p(bias), p(at), p(y), p(y), None, ROWS, 2, 0, 2, st),
            "fold-producer": lambda: L.wq4_gemm_tiled_lnfold(t.handle, p(bias), p(at), p(y), p(y), None, ROWS, 2, 0,
                                                             ctypes.byref(prod), st),
        }
        if k == 1280:
            variants["fold-consumer"] = lambda: L.wq4_gemm_tiled_lnfold(t.handle, p(bias), p(at), None, p(y), None,
                                                                        ROWS, 0, 0, ctypes.byref(cons), st)
            variants["fold-consumer-gelu-tiled"] = lambda: L.wq4_gemm_tiled_lnfold(
                t.handle, p(bias), p(at), None, None, p(yt), ROWS, 1 | 4, 0, ctypes.byref(cons), st)
        for name, fn in variants.items():
            with torch.cuda.stream(s):
                wq4.check(fn())
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(LAUNCHES):
                    wq4.check(fn())
            times = []
            for _ in range(7):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                with torch.cuda.stream(s):
                    a.record(s)
                    g.replay()
                    b.record(s)
                torch.cuda.synchronize()
                times.append(a.elapsed_time(b) * 1e3 / LAUNCHES)
            print(f"N={n:5d} K={k:5d} rows={ROWS} {name:26s}: median {np.median(times[1:]):6.2f} us/launch", flush=True)
            del g


if __name__ == "__main__":
    main()
