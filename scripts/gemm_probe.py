"""Encoder-size Q4 GEMM probe: q4_matmul at M rows over the Large-V3 encoder
shapes (N, K), REPS launches each, HIP-event timed; prints TFLOP/s per shape
(algorithmic 2 M N K).  Used under rocprofv3 (round 2; round 3: tools/enc_ab.py, scripts/gpu.sh gemm)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "whisper-burn_amd"))
import wq4  # noqa: E402

M = int(os.environ.get("ROWS", "48000"))
POLICY = int(os.environ.get("POLICY", "0"))  # kernel policy (include/wq4.h)
PREC = int(os.environ.get("PREC", "0"))  # 0 = f16x2 (default), 1 = f16
REPS = int(os.environ.get("REPS", "5"))
SHAPES = [(3840, 1280), (1280, 1280), (5120, 1280), (1280, 5120)]
rng = np.random.default_rng(0)
wq4.set_kernel_policy(POLICY)
wq4.set_precision(PREC)
for N, K in SHAPES:
    w = rng.standard_normal((N, K)).astype(np.float32) * 0.05
    t = wq4.Q4Tensor.from_q4_bytes(wq4.quantize_q4_0(w), (N, K))
    x = torch.randn(1, M, K, device="cuda")
    y = wq4.q4_matmul(x, t)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(REPS):
        y = wq4.q4_matmul(x, t)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / REPS
    print(f"N={N} K={K} M={M}: {ms:.3f} ms/call (incl. activation tiling), {2 * M * N * K / ms / 1e9:.1f} TFLOP/s", flush=True)
    del y, x
    t.close()
