"""Repeated wa_xattn_check calls at the Large-V3 decode shape, for a
rocprofv3 kernel-trace of the cross-attention kernels (xattn_q / xattn_main /
xattn_out) in isolation:

    rocprofv3 --kernel-trace --stats -d OUT -o run --output-format csv -- \
        python3 whisper-burn_amd/tools/xattn_bench.py --clips 32 --iters 20
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import numpy as np
import torch

import whisper_amd
import wq4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clips", type=int, default=32)
    ap.add_argument("--tq", type=int, default=1)
    ap.add_argument("--heads", type=int, default=20)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--f16", action="store_true")
    a = ap.parse_args()
    H, D, T = a.heads, 64 * a.heads, 1500
    rng = np.random.default_rng(0)
    enc = torch.from_numpy(rng.standard_normal((a.clips, T, D)).astype(np.float32)).cuda()
    q = torch.from_numpy(rng.standard_normal((a.clips * a.tq, D)).astype(np.float32)).cuda()
    rk = torch.from_numpy(wq4.quantize_q4_0(rng.uniform(-0.05, 0.05, (D, D)).astype(np.float32))).cuda()
    bv = torch.zeros(D, device="cuda")
    prec = wq4.PREC_F16 if a.f16 else wq4.PREC_F16X2
    for _ in range(a.iters):
        whisper_amd.xattn_check(q, rk, rk, bv, enc, a.tq, H, 0, prec)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
