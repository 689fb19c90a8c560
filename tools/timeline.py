"""Decode-step timeline of a rocprofv3 kernel trace (two decode groups on two
streams): how the groups' chains overlap.

    python tools/timeline.py <kernel_trace.csv>

Per queue: the layer period (time between consecutive xattn_main starts).
For each kernel family: mean duration, and mean duration split by whether
another queue's xattn_main was running at its midpoint.  Chip concurrency:
share of the decode window with 0 / 1 / 2+ kernels in flight.
"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
K = []
for r in rows:
    m = re.search(r"[a-z][a-z0-9]*(?:_[a-z0-9]+)*_kernel", r["Kernel_Name"])
    name = m.group(0) if m else r["Kernel_Name"][:40]
    if "q4_gemm_decode" in name or "skinny" in name:
        name = f"{name}[{r.get('Grid_Size_X', r.get('Grid_Size', ''))}]"
    K.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "0"), name))
K.sort()
dec = re.compile(r"xattn|cross_attn_kv|dec_self|q4_gemm_decode|skinny_gemm|logits_argmax|embed_fold|bookkeep")
D = [k for k in K if dec.search(k[3])]
if not D:
    sys.exit("no decode kernels")
# restrict to the decode window of the last transcribe (largest gap splits runs)
t0, t1 = D[0][0], D[-1][1]
queues = sorted({k[2] for k in D})
mains = {q: [(s, e) for s, e, qq, n in D if qq == q and n == "xattn_main_kernel"] for q in queues}
print(f"decode window {(t1 - t0) * 1e-6:.2f} ms, {len(D)} kernels on queues {queues}")
for q in queues:
    st = [s for s, _ in mains[q]]
    per = [(b - a) * 1e-3 for a, b in zip(st, st[1:]) if (b - a) < 1_000_000]
    if per:
        per.sort()
        print(f"queue {q}: {len(st)} xattn_main, layer period median {per[len(per) // 2]:.1f} us")


def other_main_running(t, q):
    for qq in queues:
        if qq == q:
            continue
        for s, e in mains[qq]:
            if s <= t <= e:
                return True
    return False


fam = collections.defaultdict(lambda: [[], []])
for s, e, q, n in D:
    fam[n][1 if other_main_running((s + e) // 2, q) else 0].append((e - s) * 1e-3)
print(f"{'kernel':48s} {'n':>6s} {'avg us':>8s} {'alone':>8s} {'n':>6s} {'beside main':>11s} {'n':>6s}")
for n, (a, b) in sorted(fam.items(), key=lambda kv: -sum(kv[1][0]) - sum(kv[1][1])):
    allv = a + b
    f = lambda v: f"{sum(v) / len(v):8.2f}" if v else "       -"
    print(f"{n[:48]:48s} {len(allv):6d} {sum(allv) / len(allv):8.2f} {f(a)} {len(a):6d} {f(b):>11s} {len(b):6d}")
# decode phases: runs of decode kernels separated by > 1 ms with none in flight
runs, cur = [], [D[0]]
for k in D[1:]:
    if k[0] - max(x[1] for x in cur[-64:]) > 1_000_000:
        runs.append(cur)
        cur = []
    cur.append(k)
runs.append(cur)
for i, run in enumerate(runs):
    ev = []
    for s, e, q, n in run:
        ev.append((s, 1))
        ev.append((e, -1))
    ev.sort()
    cnt, last = 0, ev[0][0]
    hist = collections.Counter()
    for t, d in ev:
        hist[min(cnt, 3)] += t - last
        cnt += d
        last = t
    tot = sum(hist.values())
    steps = sum(1 for k in run if k[3] == "wa28logits_argmax_f16_k32_kernel") / max(1, len(queues))
    print(f"decode run {i}: {tot * 1e-6:.2f} ms, {len(run)} kernels, ~{steps:.0f} steps per group; kernels in flight: "
          + ", ".join(f"{k if k < 3 else '3+'}: {v / tot:.1%}" for k, v in sorted(hist.items())))
# main-vs-main overlap
ov = 0
for q in queues:
    for s, e in mains[q]:
        for qq in queues:
            if qq <= q:
                continue
            for s2, e2 in mains[qq]:
                ov += max(0, min(e, e2) - max(s, s2))
tm = sum(e - s for q in queues for s, e in mains[q])
print(f"xattn_main: total {tm * 1e-6:.2f} ms of kernel time, {ov * 1e-6:.2f} ms of it with both groups' mains running")
