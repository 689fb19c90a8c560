"""Per-kernel breakdown of one decode step from a reduced rocprofv3 trace (tail.csv)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
idx = [i for i, r in enumerate(rows) if r["name"].startswith("wa::bookkeep")]
a, b = idx[-3], idx[-2]
step = rows[a:b]
t0 = int(step[0]["start"])
print(f"step wall {(int(rows[b]['start']) - t0) / 1e3:.1f} us, {len(step)} kernels, "
      f"busy {sum(int(r['end']) - int(r['start']) for r in step) / 1e3:.1f} us")
agg = {}
for r in step:
    d = agg.setdefault(r["name"][:60], [0, 0.0])
    d[0] += 1
    d[1] += (int(r["end"]) - int(r["start"])) / 1e3
for k, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{k:60s} n={c:3d} each={d / c:7.2f} us total={d:8.1f} us")
