"""Per-launch table of one decoder layer from a rocprofv3 kernel trace of a
graph-replayed decode (one decode group, e.g. `bench.py --clips-per-gpu 1`):
the launches of every layer are aligned on the layer's self-attention
launch, and per position in the layer the table gives the kernel (with its
grid), the median duration and the median gap since the previous launch
ended (the dependent-launch boundary plus whatever the launch waited on).

    python tools/layer_table.py <kernel_trace.csv> [out.json]
"""
import collections
import csv
import json
import re
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
K = []
for r in rows:
    m = re.search(r"[a-z][a-z0-9]*(?:_[a-z0-9]+)*_kernel", r["Kernel_Name"])
    name = m.group(0) if m else r["Kernel_Name"][:40]
    grid = r.get("Grid_Size_X") or r.get("Grid_Size") or ""
    wg = r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or ""
    if grid and wg:
        name = f"{name}[{int(grid) // max(1, int(wg))} wg]"
    K.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "0"), name))
K.sort()
dec = re.compile(r"xattn|cross_attn_kv|dec_self|q4_gemm_decode|skinny_gemm|logits_argmax|embed_fold|bookkeep")
D = [k for k in K if dec.search(k[3])]
if not D:
    sys.exit("no decode kernels")
q = collections.Counter(k[2] for k in D).most_common(1)[0][0]
D = [k for k in D if k[2] == q]
# layers: a self-attention launch opens position 1 of a layer (position 0 is the qkv GEMM before it)
starts = [i for i, k in enumerate(D) if "dec_self_attn" in k[3]]
layers = []
for a, b in zip(starts, starts[1:]):
    seg = D[a - 1:b - 1]
    if all(not re.search(r"logits|bookkeep|embed", k[3]) for k in seg):
        layers.append(seg)
if not layers:
    sys.exit("no whole layers found")
n = collections.Counter(len(L) for L in layers).most_common(1)[0][0]
layers = [L for L in layers if len(L) == n]
table = []
for p in range(n):
    names = collections.Counter(L[p][3] for L in layers).most_common(1)[0][0]
    durs = [(L[p][1] - L[p][0]) * 1e-3 for L in layers]
    gaps = [(L[p][0] - L[p - 1][1]) * 1e-3 for L in layers] if p > 0 else [
        (L[0][0] - prev[-1][1]) * 1e-3 for prev, L in zip(layers, layers[1:])]
    table.append({"pos": p, "kernel": names, "median_us": round(statistics.median(durs), 2),
                  "gap_before_us": round(statistics.median(gaps), 2) if gaps else None})
span = statistics.median([(L[-1][1] - L[0][0]) * 1e-3 for L in layers])
period = statistics.median([(b[0][0] - a[0][0]) * 1e-3 for a, b in zip(layers, layers[1:])])
print(f"queue {q}: {len(layers)} whole layers of {n} launches; layer period median {period:.1f} us, "
      f"first start to last end {span:.1f} us")
print(f"{'pos':>3} {'median us':>9} {'gap us':>7}  kernel")
for t in table:
    g = "" if t["gap_before_us"] is None else f"{t['gap_before_us']:7.2f}"
    print(f"{t['pos']:3d} {t['median_us']:9.2f} {g:>7}  {t['kernel']}")
busy = sum(t["median_us"] for t in table)
print(f"sum of medians {busy:.1f} us of a {period:.1f}-us layer period: {period - busy:.1f} us between launches")
if len(sys.argv) > 2:
    with open(sys.argv[2], "w") as f:
        json.dump({"queue": q, "layers": len(layers), "launches_per_layer": n, "layer_period_us": round(period, 2),
                   "table": table}, f, indent=1)
