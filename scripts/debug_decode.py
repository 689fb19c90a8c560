"""Scratch: where does the decode kernel disagree with the prefill kernel?"""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "whisper-burn_amd"))
import wq4
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "whisper-burn_amd", "tools"))
from q4_bench import rand_q4

for (m, n, k) in [(4, 64, 128), (4, 64, 1280), (4, 1280, 1280), (10, 1280, 1280)]:
    t = wq4.Q4Tensor.from_q4_bytes(rand_q4(n, k, 7), [n, k])
    x = torch.randn((1, m, k), device="cuda:0")
    wq4.set_kernel_policy(1); yp = wq4.q4_matmul(x, t).cpu().numpy().reshape(m, n)
    wq4.set_kernel_policy(2); yd = wq4.q4_matmul(x, t).cpu().numpy().reshape(m, n)
    wq4.set_kernel_policy(0)
    d = np.abs(yp - yd)
    print(f"m={m} n={n} k={k} maxdiff={d.max():.3e} rows_bad={np.where(d.max(1) > 1e-4)[0].tolist()[:12]} "
          f"cols_bad={np.where(d.max(0) > 1e-4)[0].tolist()[:12]} n_cols_bad={(d.max(0) > 1e-4).sum()}")
    if d.max() > 1e-4:
        r = int(np.argmax(d.max(1)))
        print("  row", r, "prefill", yp[r, :6], "decode", yd[r, :6])
        for rr in range(m):
            for r2 in range(m):
                if rr != r2 and np.allclose(yd[rr], yp[r2], atol=1e-4):
                    print(f"  decode row {rr} == prefill row {r2}")
