"""Why do the encoder Q4 GEMMs run slower inside the model than in
tools/pf_variants.py?  Times the four Large-V3 encoder GEMMs (M = 48000) on a
freshly tiled A operand with epilogue variants: the bare f32 store, the
model's epilogue (bias; out / fc2 + residual into x; fc1 GELU + A-tiled
output) and, for fc1, GELU alone and the A-tiled output alone.  Variants are
interleaved round by round and the minimum and median are printed (clock
ramps make single samples unreliable).
    python tools/gemm_epi_probe.py          (env: ROWS, ROUNDS, ONLY=fc1,...)
"""
import ctypes
import os
import statistics
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "whisper-burn_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))

import oracle  # noqa: E402
import wq4  # noqa: E402

M = int(os.environ.get("ROWS", "48000"))
ROUNDS = int(os.environ.get("ROUNDS", "8"))
GELU, RES, TILED = 1, 2, 4
# (name, N, K, epilogue variants: label -> flags)
SHAPES = [("qkv", 3840, 1280, {"bare": 0, "bias": 0x100}),
          ("out", 1280, 1280, {"bare": 0, "bias+res": 0x100 | RES}),
          ("fc1", 5120, 1280, {"bare": 0, "bias+gelu": 0x100 | GELU, "bias+tiled": 0x100 | TILED,
                               "bias+gelu+tiled": 0x100 | GELU | TILED}),
          ("fc2", 1280, 5120, {"bare": 0, "bias+res": 0x100 | RES})]


def main():
    L = wq4.lib()
    vp = ctypes.c_void_p
    st = vp(torch.cuda.current_stream().cuda_stream)
    rng = np.random.default_rng(0)
    only = os.environ.get("ONLY", "")
    for name, n, k, variants in SHAPES:
        if only and name not in only.split(","):
            continue
        q = oracle.quantize_convert_np((rng.standard_normal(n * k) * 0.05).astype(np.float32))
        t = wq4.Q4Tensor.from_q4_bytes(q, [n, k], decode_step=False)
        x = torch.randn(M, k, device="cuda")
        at = torch.empty(L.wq4_atiled_bytes(M, k, 0), dtype=torch.uint8, device="cuda")
        bias = torch.randn(n, device="cuda") * 0.01
        y = torch.zeros(M, n, device="cuda")
        ato = torch.empty(L.wq4_atiled_bytes(M, n, 0), dtype=torch.uint8, device="cuda")

        def tile():
            wq4.check(L.wq4_tile_activations(vp(x.data_ptr()), M, k, k, 0, vp(at.data_ptr()), at.numel(), st))

        def run(flags):
            b = vp(bias.data_ptr()) if flags & 0x100 else None
            res = vp(y.data_ptr()) if flags & RES else None
            out = None if flags & TILED else vp(y.data_ptr())
            to = vp(ato.data_ptr()) if flags & TILED else None
            wq4.check(L.wq4_gemm_tiled(t.handle, b, vp(at.data_ptr()), res, out, to, M, flags & 0xff, 0, 1, st))

        times = {lab: [] for lab in variants}
        for _ in range(ROUNDS + 1):
            for lab, flags in variants.items():
                tile()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                run(flags)
                e.record()
                torch.cuda.synchronize()
                times[lab].append(s.elapsed_time(e))
        for lab, ts in times.items():
            ts = ts[1:]  # the first round warms up
            mn, md = min(ts), statistics.median(ts)
            print(f"{name} N={n} K={k}: {lab:16s} min {mn:.4f} ms ({2 * M * n * k / mn / 1e9:6.1f} TF/s)"
                  f"  median {md:.4f} ms", flush=True)


if __name__ == "__main__":
    main()
