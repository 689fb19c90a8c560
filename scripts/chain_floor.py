"""Dispatch floor of a graph-replayed chain of trivial dependent kernels on
this box: 300 x (one-element add) captured in a torch CUDA graph and
replayed; run under rocprofv3 --kernel-trace to read each kernel's duration
and the gaps (scripts/trace_gaps.py).  Compares with the decode step's
kernel durations."""
import time

import torch

x = torch.zeros(1, device="cuda")
s = torch.cuda.Stream()
torch.cuda.synchronize()
with torch.cuda.stream(s):
    for _ in range(3):
        x.add_(1.0)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(300):
            x.add_(1.0)
torch.cuda.synchronize()
for _ in range(5):
    g.replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    g.replay()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 20
print(f"300-kernel graph replay: {dt * 1e6:.1f} us = {dt / 300 * 1e6:.2f} us per dependent kernel")
