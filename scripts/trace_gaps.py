"""Launch-chain gaps from a rocprofv3 kernel_trace.csv (one decode group).

usage: trace_gaps.py <kernel_trace.csv> [out.json]
Per queue, kernels sorted by start: gap = start(i+1) - end(i). Reports, for
the decode kernels (the graph-replayed step), the mean busy time and mean gap
per kernel family -- how much of a step is kernel execution and how much is
the dependency/launch latency between kernels.
"""
import collections
import csv
import json
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
byq = collections.defaultdict(list)
for r in rows:
    m = re.search(r"[a-z][a-z0-9]*(?:_[a-z0-9]+)*_kernel", r["Kernel_Name"])
    name = m.group(0) if m else r["Kernel_Name"][:40]
    byq[r.get("Queue_Id", "0")].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
dur = collections.defaultdict(list)
gap = collections.defaultdict(list)
decode = re.compile(r"xattn|dec_self|q4_gemm_decode|skinny_gemm|logits_argmax|embed_fold|bookkeep")
for q, ks in byq.items():
    ks.sort()
    for i in range(1, len(ks)):
        s, e, n = ks[i]
        if not decode.search(n):
            continue
        g = s - ks[i - 1][1]
        if 0 <= g < 100_000:  # same-chain successor (skip host waits between steps)
            dur[n].append((e - s) * 1e-3)
            gap[n].append(g * 1e-3)
out = {}
tb = tg = 0.0
for n in sorted(dur, key=lambda n: -sum(dur[n])):
    d, g = dur[n], gap[n]
    out[n] = {"launches": len(d), "avg_us": round(sum(d) / len(d), 2), "avg_gap_before_us": round(sum(g) / len(g), 2)}
    tb += sum(d)
    tg += sum(g)
    print(f"{n:28s} n={len(d):6d} busy={sum(d) / len(d):7.2f}us gap_before={sum(g) / len(g):6.2f}us")
print(f"decode kernels: busy {tb / 1e3:.1f} ms, gaps {tg / 1e3:.1f} ms ({100 * tg / max(tb + tg, 1e-9):.1f} % of the chain)")
if len(sys.argv) > 2:
    json.dump({"per_kernel": out, "busy_ms": tb / 1e3, "gap_ms": tg / 1e3}, open(sys.argv[2], "w"), indent=1)
