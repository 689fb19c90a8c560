"""A/B timing of prefill-GEMM builds in ONE process (cdna_hip_programming.md
§5.4 rule 24): each libwq4.so given on the command line is loaded RTLD_LOCAL,
and the four Large-V3 encoder GEMM shapes are timed on each, interleaved over
ROUNDS rounds, on the same random operands.  Prints per (lib, shape) the
median / min ms and TFLOP/s (algorithmic 2 M N K).

    python tools/pf_variants.py lib/libwq4.so diag/pf1/libwq4.so ...
    env: ROWS (default 48000), ROUNDS (5), REPS (5 launches per timing)
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "whisper-burn_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))

M = int(os.environ.get("ROWS", "48000"))
ROUNDS = int(os.environ.get("ROUNDS", "5"))
REPS = int(os.environ.get("REPS", "5"))
SHAPES = [(3840, 1280), (1280, 1280), (5120, 1280), (1280, 5120)]
vp = ctypes.c_void_p


def load(path):
    L = ctypes.CDLL(os.path.abspath(path), mode=os.RTLD_LOCAL | os.RTLD_NOW)
    L.wq4_tensor_create.argtypes = [ctypes.c_int, vp, ctypes.c_size_t, ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(vp)]
    L.wq4_gemm_tiled.argtypes = [vp, vp, vp, vp, vp, vp, ctypes.c_int64, ctypes.c_uint, ctypes.c_int, ctypes.c_int, vp]
    L.wq4_tile_activations.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, vp, ctypes.c_size_t, vp]
    L.wq4_atiled_bytes.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
    L.wq4_atiled_bytes.restype = ctypes.c_size_t
    L.wq4_last_error.restype = ctypes.c_char_p
    return L


def chk(L, rc):
    if rc != 0:
        raise RuntimeError(L.wq4_last_error().decode())


def main():
    import oracle

    libs = sys.argv[1:] or ["whisper-burn_amd/lib/libwq4.so"]
    Ls = [load(p) for p in libs]
    mode = os.environ.get("ENC_MODE")  # wq4_debug_set_enc_kernel in every lib (ring-kernel geometry)
    if mode is not None:
        for L in Ls:
            if hasattr(L, "wq4_debug_set_enc_kernel"):
                L.wq4_debug_set_enc_kernel(int(mode))
    rng = np.random.default_rng(0)
    st = vp(torch.cuda.current_stream().cuda_stream)
    setups = []
    for n, k in SHAPES:
        q = oracle.quantize_convert_np((rng.standard_normal(n * k) * 0.05).astype(np.float32))
        x = torch.randn(M, k, device="cuda")
        y = torch.empty(M, n, device="cuda")
        per = []
        for L in Ls:
            h = vp()
            chk(L, L.wq4_tensor_create(0, q.ctypes.data, q.size, n, k, ctypes.byref(h)))
            atb = L.wq4_atiled_bytes(M, k, 0)
            at = torch.empty(atb, dtype=torch.uint8, device="cuda")
            chk(L, L.wq4_tile_activations(vp(x.data_ptr()), M, k, k, 0, vp(at.data_ptr()), atb, st))
            per.append((h, at))
        setups.append((n, k, y, per))
    torch.cuda.synchronize()
    times = {(li, si): [] for li in range(len(Ls)) for si in range(len(SHAPES))}
    outs = {}
    for r in range(ROUNDS):
        for si, (n, k, y, per) in enumerate(setups):
            for li, L in enumerate(Ls):
                h, at = per[li]
                run = lambda: chk(L, L.wq4_gemm_tiled(h, None, vp(at.data_ptr()), None, vp(y.data_ptr()), None, M, 0, 0, 1, st))
                run()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(REPS):
                    run()
                e.record()
                torch.cuda.synchronize()
                times[(li, si)].append(s.elapsed_time(e) / REPS)
                if r == 0:
                    outs[(li, si)] = y[:64].clone()
    for si, (n, k, _, _) in enumerate(setups):
        for li, p in enumerate(libs):
            t = np.array(times[(li, si)])
            same = bool(torch.equal(outs[(li, si)], outs[(0, si)]))
            print(f"N={n:5d} K={k:5d} M={M} {p:40s} median {np.median(t):.4f} ms min {t.min():.4f} "
                  f"-> {2 * M * n * k / np.median(t) / 1e9:7.1f} TF/s  (bits == lib0: {same})", flush=True)


if __name__ == "__main__":
    main()
