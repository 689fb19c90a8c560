"""Average kernel durations from a rocprofv3 kernel_trace.csv, split by grid size.

usage: trace_by_grid.py <kernel_trace.csv> <name-regex> [out.json]
The bench's HIP-event probe launches the decode cross-attention at all clips of
the batch in one launch, while the graph-replayed decode runs it per decode
group: the two shapes have different grids, so this separates them and gives
the rocprof duration to compare with bench.py's roofline avg_us.
"""
import collections
import csv
import json
import re
import sys

path, rx = sys.argv[1], re.compile(sys.argv[2])
agg = collections.defaultdict(list)
for r in csv.DictReader(open(path)):
    name = r.get("Kernel_Name", "")
    if not rx.search(name):
        continue
    grid = tuple(int(r[k]) for k in sorted(r) if k.startswith("Grid_Size") and r[k] != "")
    wg = tuple(int(r[k]) for k in sorted(r) if k.startswith("Workgroup_Size") and r[k] != "")
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
    m = re.search(r"[a-z][a-z0-9]*(?:_[a-z0-9]+)*_kernel", name)
    short = m.group(0) if m else name[:60]
    agg[(short, grid, wg)].append(dur)
out = []
for (name, grid, wg), v in sorted(agg.items()):
    v.sort()
    out.append({"kernel": name, "grid": grid, "workgroup": wg, "launches": len(v),
                "avg_us": round(sum(v) / len(v), 2), "median_us": round(v[len(v) // 2], 2)})
    print(f"{name:28s} grid={grid} wg={wg} n={len(v):6d} avg={sum(v) / len(v):8.2f}us median={v[len(v) // 2]:8.2f}us")
if len(sys.argv) > 3:
    json.dump(out, open(sys.argv[3], "w"), indent=1)
