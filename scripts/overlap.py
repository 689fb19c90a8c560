"""Concurrency in a reduced rocprofv3 trace (tail.csv): busy-union vs sum of kernel durations."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["start"]), int(r["end"]), r["name"]) for r in rows)
t0, t1 = iv[0][0], max(e for _, e, _ in iv)
tot = sum(e - s for s, e, _ in iv)
union, cs, ce = 0, None, None
for s, e, _ in iv:
    if cs is None or s > ce:
        if cs is not None:
            union += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
union += ce - cs
print(f"window {(t1 - t0) / 1e3:.0f} us, kernels {len(iv)}, sum {tot / 1e3:.0f} us, union {union / 1e3:.0f} us, "
      f"overlap factor {tot / union:.2f}")
# overlap by kernel kind: how often a kernel of kind X runs beside another kernel
