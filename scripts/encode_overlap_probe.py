"""Can the next batch's encoder run beside a decode on a CU-masked stream?

Model A transcribes 32 clips (encoder + two-group decode, fixed 224 steps);
model B runs encoders back to back in a second thread on a stream created by
hipExtStreamCreateWithCUMask.  Prints: B's encoder alone at each mask (does
the mask restrict it?), A alone, then A's decode with B encoding beside it
and the encoders B finished meanwhile.
    python3 scripts/encode_overlap_probe.py [N ...]     (mask sizes, CUs)
MASK=stride -> the N CUs are spread (bit i * 256 / N) instead of bits 0..N-1.
"""
import ctypes
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "whisper-burn_amd")]
import torch  # noqa: E402

import whisper_amd  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")


def masked_stream(n, total=256):
    words = (ctypes.c_uint32 * (total // 32))()
    bits = [i * total // n for i in range(n)] if os.environ.get("MASK") == "stride" else range(n)
    for i in bits:
        words[i // 32] |= 1 << (i % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(total // 32), words)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value)


sizes = [int(x) for x in sys.argv[1:]] or [32, 64, 128]
B = 32
A = whisper_amd.WhisperModel("large_v3", 1234, max_batch=B)
Bm = whisper_amd.WhisperModel("large_v3", 99, max_batch=B)
g = torch.Generator(device="cuda").manual_seed(0)
mel = torch.randn((B, 128, 3000), device="cuda", generator=g) * 0.5
streams = {n: masked_stream(n) for n in sizes}


def enc_time(s, k=2):
    with torch.cuda.stream(s):
        Bm.encode(mel)
        s.synchronize()
        t = time.perf_counter()
        for _ in range(k):
            Bm.encode(mel)
        s.synchronize()
    return (time.perf_counter() - t) / k * 1e3


for n in sizes:
    print("B encoder alone, mask %d CUs: %.1f ms" % (n, enc_time(streams[n])), flush=True)
A.transcribe(mel, max_tokens=224, eot_stop=False)
A.transcribe(mel, max_tokens=224, eot_stop=False)
print("A alone", A.last_timings(), flush=True)
for n in sizes:
    stop = threading.Event()
    done = []

    def worker(s=streams[n]):
        with torch.cuda.stream(s):
            while not stop.is_set():
                t = time.perf_counter()
                Bm.encode(mel)
                s.synchronize()
                done.append((time.perf_counter() - t) * 1e3)

    th = threading.Thread(target=worker)
    th.start()
    time.sleep(0.5)
    A.transcribe(mel, max_tokens=224, eot_stop=False)
    tA = A.last_timings()
    stop.set()
    th.join()
    print("mask %d: A with B encoding %s; B encoders %d, ms %s" % (n, tA, len(done), [round(x) for x in done]),
          flush=True)
