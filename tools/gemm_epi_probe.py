"""Why do the encoder Q4 GEMMs run slower inside the model than in
tools/pf_variants.py?  Times the four Large-V3 encoder GEMMs (M = 48000) with
(a) the bare f32 epilogue on a warm operand (pf_variants' setting), (b) the
model's epilogue (bias; out / fc2 + residual into x; fc1 GELU + A-tiled
output), (c) as (b) with the A operand rewritten by a tiling pass right before
every launch (a freshly produced operand, as the LayerNorm leaves it).
    python tools/gemm_epi_probe.py          (env: ROWS, REPS)
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

M = int(os.environ.get("ROWS", "48000"))
REPS = int(os.environ.get("REPS", "5"))
GELU, RES, TILED = 1, 2, 4
# (name, N, K, flags of the model's launch)
SHAPES = [("qkv", 3840, 1280, 0), ("out", 1280, 1280, RES), ("fc1", 5120, 1280, GELU | TILED), ("fc2", 1280, 5120, RES)]


def main():
    L = wq4.lib()
    vp = ctypes.c_void_p
    st = vp(torch.cuda.current_stream().cuda_stream)
    rng = np.random.default_rng(0)
    for name, n, k, flags in SHAPES:
        q = oracle.quantize_convert_np((rng.standard_normal(n * k) * 0.05).astype(np.float32))
        t = wq4.Q4Tensor.from_q4_bytes(q, [n, k], decode_step=False)
        x = torch.randn(M, k, device="cuda")
        at = torch.empty(L.wq4_atiled_bytes(M, k, 0), dtype=torch.uint8, device="cuda")
        tile = lambda: wq4.check(L.wq4_tile_activations(vp(x.data_ptr()), M, k, k, 0, vp(at.data_ptr()), at.numel(), st))
        tile()
        bias = torch.randn(n, device="cuda") * 0.01
        y = torch.zeros(M, n, device="cuda")
        ato = torch.empty(L.wq4_atiled_bytes(M, n, 0), dtype=torch.uint8, device="cuda")

        def bare():
            wq4.check(L.wq4_gemm_tiled(t.handle, None, vp(at.data_ptr()), None, vp(y.data_ptr()), None, M, 0, 0, 1, st))

        def model():
            res = vp(y.data_ptr()) if flags & RES else None
            out = None if flags & TILED else vp(y.data_ptr())
            to = vp(ato.data_ptr()) if flags & TILED else None
            wq4.check(L.wq4_gemm_tiled(t.handle, vp(bias.data_ptr()), vp(at.data_ptr()), res, out, to, M, flags, 0, 1,
                                       st))

        def timed(fn, fresh):
            fn()
            tot = 0.0
            for _ in range(REPS):
                if fresh:
                    tile()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                fn()
                e.record()
                torch.cuda.synchronize()
                tot += s.elapsed_time(e)
            return tot / REPS

        for label, fn, fresh in (("bare, warm A", bare, False), ("model epilogue, warm A", model, False),
                                 ("model epilogue, fresh A", model, True), ("bare, fresh A", bare, True)):
            ms = timed(fn, fresh)
            print(f"{name} N={n} K={k}: {label:24s} {ms:.4f} ms  {2 * M * n * k / ms / 1e9:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
