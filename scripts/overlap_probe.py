"""Can the next batch's encoder run beside a decode?  Model A transcribes 32
clips (encoder + two-group decode) while model B, on its own CU-masked
stream (WA_ENC_CU_MASK=N at its creation), runs encoders back to back in a
second thread.  Prints A's phase times alone and with B running, and B's
encoder time alone and under A's decode.   python3 scripts/overlap_probe.py N
(WA_ENC_CU_MASK lived in the r02 experiment build of wa_model.cpp only: the
mask did not restrict the encoder, DESIGN.md §4 dead ends.)"""
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "whisper-burn_amd"), os.path.join(REPO, "oracle")]
import torch  # noqa: E402

import whisper_amd  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 64
B = 32
A = whisper_amd.WhisperModel("large_v3", 1234, max_batch=B)
os.environ["WA_ENC_CU_MASK"] = str(N)
Bm = whisper_amd.WhisperModel("large_v3", 99, max_batch=B)
os.environ.pop("WA_ENC_CU_MASK")
g = torch.Generator(device="cuda").manual_seed(0)
mel = torch.randn((B, 128, 3000), device="cuda", generator=g) * 0.5
s2 = torch.cuda.Stream()


def enc_time(k=3):
    with torch.cuda.stream(s2):
        Bm.encode(mel)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(k):
            Bm.encode(mel)
        torch.cuda.synchronize()
    return (time.perf_counter() - t) / k * 1e3


A.transcribe(mel, max_tokens=224, eot_stop=False)
print("A alone", A.last_timings(), flush=True)
print("B encoder alone (masked %d CUs): %.1f ms" % (N, enc_time()), flush=True)
stop = threading.Event()
done = []


def worker():
    with torch.cuda.stream(s2):
        while not stop.is_set():
            t = time.perf_counter()
            Bm.encode(mel)
            s2.synchronize()
            done.append((time.perf_counter() - t) * 1e3)


th = threading.Thread(target=worker)
th.start()
time.sleep(0.3)
A.transcribe(mel, max_tokens=224, eot_stop=False)
tA = A.last_timings()
stop.set()
th.join()
print("A with B encoding", tA, flush=True)
print("B encoders during A: %d, ms each %s" % (len(done), [round(x, 1) for x in done]), flush=True)
