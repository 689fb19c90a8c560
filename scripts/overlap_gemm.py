"""Scratch: do decode-GEMM graphs on two streams overlap?"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "whisper-burn_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "whisper-burn_amd", "tools"))
import wq4  # noqa: E402
from q4_bench import rand_q4  # noqa: E402

L = wq4.lib()
m, n, k, P = 32, 1280, 1280, wq4.PREC_F16X2
ts = [wq4.Q4Tensor.from_q4_bytes(rand_q4(n, k, i), [n, k]) for i in range(2)]
graphs = []
streams = [torch.cuda.Stream() for _ in range(2)]
for i, s in enumerate(streams):
    x = torch.randn((m, k), device="cuda:0")
    atb = L.wq4_atiled_bytes(m, k, P)
    at = torch.empty(atb, dtype=torch.uint8, device="cuda:0")
    y = torch.empty((m, n), device="cuda:0")
    with torch.cuda.stream(s):
        st = ctypes.c_void_p(s.cuda_stream)
        wq4.check(L.wq4_tile_activations(ctypes.c_void_p(x.data_ptr()), m, k, k, P, ctypes.c_void_p(at.data_ptr()), atb, st))
        run = lambda: wq4.check(L.wq4_gemm_tiled(ts[i].handle, None, ctypes.c_void_p(at.data_ptr()), None,  # noqa: E731
                                                 ctypes.c_void_p(y.data_ptr()), None, m, 0, P, 2, st))
        run()
        s.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(100):
                run()
        graphs.append((g, x, at, y))
torch.cuda.synchronize()
for ns in (1, 2):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for i in range(ns):
        streams[i].wait_event(e0)
        with torch.cuda.stream(streams[i]):
            for _ in range(3):
                graphs[i][0].replay()
    for i in range(ns):
        torch.cuda.current_stream().wait_stream(streams[i])
    e1.record()
    torch.cuda.synchronize()
    print(f"{ns} stream(s): {e0.elapsed_time(e1) * 1e3 / 300:.2f} us per GEMM per stream")
