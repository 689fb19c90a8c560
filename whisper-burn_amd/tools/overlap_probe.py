"""Probe: does an encoder pass on another stream slow the latency-bound decode?

Model A transcribes 32 clips (fixed length) while model B runs encoder passes
back to back on its own stream (a second replica: weights are small).  Prints
A's time alone and under load, and the encoder passes B finished meanwhile.
"""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

import whisper_amd  # noqa: E402

TOK = int(os.environ.get("TOK", "64"))
B = 32
a = whisper_amd.WhisperModel("large_v3", 1234, max_batch=B)
b = whisper_amd.WhisperModel("large_v3", 1234, max_batch=B)
mel = torch.rand((B, 128, 3000), device="cuda") * 2.5 - 1.5
CUMASK = os.environ.get("CUMASK")  # e.g. 0000ffff: CUs bits per 32-bit word, 8 words
if CUMASK:
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so")
    words = (ctypes.c_uint32 * 8)(*([int(CUMASK, 16)] * 8))
    sp = ctypes.c_void_p()
    assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(sp), 8, words) == 0
    sb = torch.cuda.ExternalStream(sp.value)
else:
    sb = torch.cuda.Stream(priority=int(os.environ.get("PRIO", "0")))
a.transcribe(mel, max_tokens=TOK, eot_stop=False)
with torch.cuda.stream(sb):
    b.encode(mel)
torch.cuda.synchronize()


def run_a():
    t0 = time.perf_counter()
    a.transcribe(mel, max_tokens=TOK, eot_stop=False)
    return time.perf_counter() - t0


ta = min(run_a() for _ in range(2))
with torch.cuda.stream(sb):
    t0 = time.perf_counter()
    b.encode(mel)
    sb.synchronize()
    te = time.perf_counter() - t0
stop = threading.Event()
count = [0]


def loop_b():
    with torch.cuda.stream(sb):
        while not stop.is_set():
            b.encode(mel)
            sb.synchronize()
            count[0] += 1


th = threading.Thread(target=loop_b)
th.start()
time.sleep(0.05)
tl = run_a()
stop.set()
th.join()
print(f"A transcribe alone {ta * 1e3:.1f} ms, under encoder load {tl * 1e3:.1f} ms; "
      f"B encoder alone {te * 1e3:.1f} ms, passes during A: {count[0]}")
