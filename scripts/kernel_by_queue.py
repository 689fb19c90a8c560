"""Per-queue launch statistics of the kernels matching a regex, from a
rocprofv3 kernel trace (csv): the pipelined bench runs the next batch's
first encoder layers on a CU-masked stream (32 CUs) beside the decode, so
rocprofv3's per-kernel average mixes those slow launches with the
full-width ones that bench.py's `roofline_q4_gemm` times (HIP events on the
model stream only).  Split by queue the two can be compared.

    python scripts/kernel_by_queue.py <kernel_trace.csv> <regex> [out.json]
"""
import collections
import csv
import json
import re
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pat = re.compile(sys.argv[2])
by = collections.defaultdict(list)
for r in rows:
    name = r["Kernel_Name"]
    if not pat.search(name):
        continue
    m = re.search(r"[a-z][a-z0-9]*(?:_[a-z0-9]+)*_kernel(?:I[^E]*E)?", name)
    short = m.group(0) if m else name[:60]
    by[(short, r.get("Queue_Id", "?"))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
out = []
for (k, q), d in sorted(by.items()):
    out.append({"kernel": k, "queue": q, "launches": len(d), "avg_us": round(statistics.mean(d), 2),
                "median_us": round(statistics.median(d), 2), "min_us": round(min(d), 2), "max_us": round(max(d), 2),
                "sum_ms": round(sum(d) * 1e-3, 3)})
    print(f"{k:45s} queue {q:>3s}: {len(d):5d} launches, avg {statistics.mean(d):9.2f} us, "
          f"median {statistics.median(d):9.2f}, sum {sum(d) * 1e-3:8.2f} ms")
if len(sys.argv) > 3:
    json.dump(out, open(sys.argv[3], "w"), indent=1)
