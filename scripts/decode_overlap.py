"""Wall-time view of the decode from a rocprofv3 kernel trace of bench.py
(scripts/gpu.sh trace): two decode groups replay their step graphs on two
streams, so summed kernel time over-counts the wall clock wherever kernels of
both groups run at once.

    python3 scripts/decode_overlap.py <kernel_trace.csv[.gz]> <variant> <weights> <precision> <clips> <out.json>

Per kernel family inside the last decode run (the timed transcribe): launches,
summed kernel time, the UNION of its intervals (wall time during which at
least one of its launches runs on either group) and union / sum.  For
xattn_main also the concurrent streaming rate: algorithmic bytes of all its
launches (each reads the encoder-output planes of its group's clips, f16 hi
and lo, + raw Wk, Wv + operands; bench.py's figure per launch) over the union.
bench.py scales its summed-GPU-time figures by union / sum so the dominant
kernel is chosen by wall-time share, like for like with the serial encoder
GEMMs.
"""
import collections
import csv
import gzip
import json
import re
import sys

path, variant, weights, prec, clips, out = sys.argv[1:7]
op = gzip.open if path.endswith(".gz") else open
rows = list(csv.DictReader(op(path, "rt")))
K = []
for r in rows:
    m = re.search(r"[a-z][a-z0-9]*(?:_[a-z0-9]+)*_kernel", r["Kernel_Name"])
    name = m.group(0) if m else r["Kernel_Name"][:40]
    grid = tuple(int(r[k]) for k in sorted(r) if k.startswith("Grid_Size") and r[k] != "")
    K.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, grid))
K.sort()
dec = re.compile(r"xattn|cross_attn_kv|dec_self|q4_gemm_decode|skinny_gemm|logits_argmax|embed_fold|bookkeep")
D = [k for k in K if dec.search(k[2])]
if not D:
    sys.exit("no decode kernels in the trace")
# decode runs: separated by > 1 ms with no decode kernel in flight; keep the last long one
runs, cur, end = [], [D[0]], D[0][1]
for k in D[1:]:
    if k[0] - end > 1_000_000:
        runs.append(cur)
        cur = []
    cur.append(k)
    end = max(end, k[1])
runs.append(cur)
run = max(runs[-2:], key=len) if len(runs) > 1 else runs[-1]
t0, t1 = run[0][0], max(k[1] for k in run)


def family(name: str) -> str:
    if name.startswith("xattn") or name.startswith("cross_attn_kv"):
        return "cross_attention"
    if "q4_gemm_decode" in name or "skinny" in name:
        return "decode_gemm"
    if "dec_self" in name:
        return "self_attention"
    if "logits" in name:
        return "logits"
    return "other"


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot


groups = collections.defaultdict(list)
for s, e, n, g in run:
    groups[family(n)].append((s, e))
    groups[n].append((s, e))
fam = {}
for key, iv in sorted(groups.items()):
    su, un = sum(e - s for s, e in iv), union(iv)
    fam[key] = {"launches": len(iv), "sum_us": round(su * 1e-3, 1), "union_us": round(un * 1e-3, 1),
                "union_over_sum": round(un / su, 4) if su else None, "wall_share": round(un / (t1 - t0), 4)}
res = {"workload": {"variant": variant, "weights": weights, "precision": prec, "clips": int(clips)},
       "source": "rocprofv3 --kernel-trace of bench.py (scripts/gpu.sh trace; decode graphs replayed), last decode run",
       "decode_window_us": round((t1 - t0) * 1e-3, 1), "kernels_in_run": len(run), "families": fam}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "families"}))
for k, v in fam.items():
    print(f"{k:40s} {v}")
