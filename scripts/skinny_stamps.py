"""Phase timing of the decode-step GEMM from its in-kernel stamps (WQ4_STAMP
build: make -C whisper-burn_amd stamp; run with WQ4_LIB_DIR=.../diag/stamp),
or, with GETTER=decode, of the 8-wave decode kernel the model runs by
default (make -C whisper-burn_amd variant V=stamp DEFS=-DWQ4_STAMP=1,
WQ4_LIB_DIR=.../diag/stamp).

Decodes one group of 32 Large-V3 clips for a few steps, then, per GEMM shape
(N, K), averages over the graph-replayed launches of the last step:
start skew of the workgroups, time to the first unit's operands, the MFMA
loop, the reduction barrier, the epilogue, and the kernel span (first start
to last end), all in microseconds (s_memrealtime, 100 MHz)."""
import collections
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "whisper-burn_amd"))
import whisper_amd  # noqa: E402
import wq4  # noqa: E402

B = int(os.environ.get("CLIPS", "32"))
m = whisper_amd.WhisperModel("large_v3", 1234, max_batch=B)
mel = torch.from_numpy(np.stack([whisper_amd.synth_uniform(0x5EED0000 + c, "mel", 128 * 3000, -1.5, 1.0)
                                 for c in range(B)]).reshape(B, 128, 3000)).cuda()
m.transcribe(mel, 50259, 8, eot_stop=False)
torch.cuda.synchronize()
L = wq4.lib()
DECODE = os.environ.get("GETTER") == "decode"
get = L.wq4_diag_decode_stamps if DECODE else L.wq4_diag_skinny_stamps
get.restype = ctypes.c_int
NL, NW, NS = 512, (256 if DECODE else 512), 8
buf = np.zeros(NL * NW * NS, np.uint64)
meta = np.zeros(NL * 3, np.int32)
n = get(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)),
                             meta.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), NL)
print("stamped launches", n)
buf = buf.reshape(NL, NW, NS).astype(np.int64)
meta = meta.reshape(NL, 3)
agg = collections.defaultdict(list)
for i in range(n):
    N, K, rows = meta[i]
    s = buf[i][buf[i, :, 0] > 0]  # workgroups that stamped (split-K: the last arriver of each tile)
    if len(s) == 0:
        continue
    t0 = s[:, 0].min()
    us = lambda a: (a - t0) * 0.01  # noqa: E731  (100 MHz)
    agg[(N, K, rows)].append([len(s), np.mean(us(s[:, 0])), np.mean(s[:, 1] - s[:, 0]) * 0.01,
                              np.mean(s[:, 2] - s[:, 1]) * 0.01, np.mean(s[:, 3] - s[:, 2]) * 0.01,
                              np.mean(s[:, 4] - s[:, 3]) * 0.01, us(s[:, 4].max()), np.mean(s[:, 6] - s[:, 5])])
print(f"{'N':>6} {'K':>6} {'rows':>4} {'n':>4} {'wgs':>4} | start-skew  loads  mfma  reduce  epilogue | span(us)  cycles")
for (N, K, rows), v in sorted(agg.items()):
    a = np.mean(np.array(v), axis=0)
    print(f"{N:6d} {K:6d} {rows:4d} {len(v):4d} {a[0]:4.0f} | {a[1]:9.2f} {a[2]:6.2f} {a[3]:5.2f} {a[4]:7.2f} "
          f"{a[5]:9.2f} | {a[6]:8.2f} {a[7]:7.0f}")
