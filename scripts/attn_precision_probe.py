"""Where does the f16x2 encoder attention lose precision?  Error vs float64
for scaled inputs (diagnostic; prints one line per variant)."""
import sys
import numpy as np
import torch
sys.path.insert(0, "whisper-burn_amd")
sys.path.insert(0, "tests")
import whisper_amd
from test_kernels_gpu import _sdpa64

T, H = 1500, 1
D = 64 * H
rng = np.random.default_rng(1)
base = rng.standard_normal((T, 3 * D)).astype(np.float32)
for name, qs, ks, vs in [("q2", 2, 1, 1), ("q0", 0, 1, 1), ("q2_v64", 2, 1, 64), ("q2_v1/1024", 2, 1, 1 / 1024),
                         ("q8", 8, 1, 1), ("q0.25", 0.25, 1, 1), ("q2_k64", 2 / 64, 64, 1), ("q128_k1/64", 128, 1 / 64, 1)]:
    x = base.copy()
    x[:, :D] *= qs
    x[:, D:2 * D] *= ks
    x[:, 2 * D:] *= vs
    out = whisper_amd.encoder_attention_check(torch.from_numpy(x).cuda(), T, H).cpu().numpy()
    ref = _sdpa64(x[:, :D], x[:, D:2 * D], x[:, 2 * D:])
    # f32 numpy reference (the oracle's arithmetic) for scale
    s = (x[:, :D] @ x[:, D:2 * D].T) / np.float32(8)
    s = s - s.max(-1, keepdims=True)
    p = np.exp(s)
    p /= p.sum(-1, keepdims=True)
    r32 = p @ x[:, 2 * D:]
    vmax = np.abs(x[:, 2 * D:]).max()
    print(f"{name:12s} gpu err/max|v| {np.abs(out - ref).max() / vmax:.3e}   f32 err/max|v| {np.abs(r32 - ref).max() / vmax:.3e}",
          flush=True)
