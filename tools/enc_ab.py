"""A/B timing of the encoder-size Q4 GEMM kernels in ONE process
(cdna_hip_programming.md §5.4 rule 24): the prefill tile kernel (mode 0)
against the LDS-DMA ring kernel's two geometries (2: 256 x 256, 3: 64 x 128),
switched with wq4_debug_set_enc_kernel, on the four Large-V3 encoder shapes,
interleaved over ROUNDS rounds on the same random operands.  Prints median /
min ms and algorithmic TFLOP/s (2 M N K) per (shape, mode).

    ROWS=48000 python tools/enc_ab.py      (env: ROWS, ROUNDS, REPS, MODES, FLAGS)

FLAGS (the encoder's epilogues): 0 f32 rows, 2 + residual (in place: out and
fc2), 5 GELU into the next GEMM's A-tiled operand (fc1), 1 | 4 alone as in
test_enc_kernel_bit_identical.
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
ROUNDS = int(os.environ.get("ROUNDS", "5"))
REPS = int(os.environ.get("REPS", "5"))
MODES = [int(v) for v in os.environ.get("MODES", "0,2,3").split(",")]
SHAPES = [(3840, 1280), (1280, 1280), (5120, 1280), (1280, 5120)]
FLAGS = int(os.environ.get("FLAGS", "0"))


def masked_stream(n):
    """MASK_CUS=n: a stream on CU-mask bits 0..n-1 (n / 8 CUs of every XCD),
    the pipelined transcribe's encoder stream."""
    hip = ctypes.CDLL("libamdhip64.so")
    words = (ctypes.c_uint32 * 8)()
    for i in range(n):
        words[i // 32] |= 1 << (i % 32)
    s = ctypes.c_void_p()
    assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(8), words) == 0
    return torch.cuda.ExternalStream(s.value)


def main():
    if os.environ.get("MASK_CUS"):
        with torch.cuda.stream(masked_stream(int(os.environ["MASK_CUS"]))):
            return run_all()
    return run_all()


def run_all():
    L = wq4.lib()
    vp = ctypes.c_void_p
    st = vp(torch.cuda.current_stream().cuda_stream)
    rng = np.random.default_rng(0)
    setups = []
    for n, k in SHAPES:
        q = oracle.quantize_convert_np((rng.standard_normal(n * k) * 0.05).astype(np.float32))
        t = wq4.Q4Tensor.from_q4_bytes(q, [n, k], decode_step=False)
        x = torch.randn(M, k, device="cuda")
        at = torch.empty(L.wq4_atiled_bytes(M, k, 0), dtype=torch.uint8, device="cuda")
        wq4.check(L.wq4_tile_activations(vp(x.data_ptr()), M, k, k, 0, vp(at.data_ptr()), at.numel(), st))
        y = torch.zeros(M, n, device="cuda")
        ot = torch.empty(L.wq4_atiled_bytes(M, n, 0), dtype=torch.uint8, device="cuda") if FLAGS & 4 else None
        setups.append((n, k, t, at, y, ot))
    torch.cuda.synchronize()
    times = {}
    prev = L.wq4_debug_set_enc_kernel(1)
    for _ in range(ROUNDS):
        for si, (n, k, t, at, y, ot) in enumerate(setups):
            for mode in MODES:
                L.wq4_debug_set_enc_kernel(mode)
                res = vp(y.data_ptr()) if FLAGS & 2 else None
                out = None if FLAGS & 4 else vp(y.data_ptr())
                tout = vp(ot.data_ptr()) if ot is not None else None
                run = lambda: wq4.check(L.wq4_gemm_tiled(t.handle, None, vp(at.data_ptr()), res, out, tout,
                                                         M, FLAGS, 0, 1, st))
                run()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(REPS):
                    run()
                e.record()
                torch.cuda.synchronize()
                times.setdefault((si, mode), []).append(s.elapsed_time(e) / REPS)
    L.wq4_debug_set_enc_kernel(prev)
    for si, (n, k, *_rest) in enumerate(setups):
        for mode in MODES:
            a = np.array(times[(si, mode)])
            print(f"N={n:5d} K={k:5d} M={M} flags {FLAGS} mode {mode}: median {np.median(a):.4f} ms min {a.min():.4f} "
                  f"-> {2 * M * n * k / np.median(a) / 1e9:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
