"""Print the top kernels of a rocprofv3 --stats kernel_stats.csv (time share)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f'{r["Name"][:80]:80s} {r["Calls"]:>7} {float(r["AverageNs"]) / 1e3:9.2f}us '
          f'{float(r["TotalDurationNs"]) / 1e6:9.1f}ms {100 * float(r["TotalDurationNs"]) / tot:5.1f}%')
print(f"total {tot / 1e6:.1f} ms")
