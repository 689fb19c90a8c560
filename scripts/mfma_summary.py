"""Summarise a rocprofv3 --pmc counter CSV of the prefill GEMM: per grid,
MFMA-busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 256 CUs
x 4 SIMDs), effective clock, and the wave-state split."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
f = (glob.glob(f"{d}/*/run_counter_collection.csv") + glob.glob(f"{d}/run_counter_collection.csv"))[0]
per = collections.defaultdict(lambda: collections.defaultdict(float))
dur = {}
for row in csv.DictReader(open(f)):
    key = (row["Kernel_Name"][:40], row.get("Grid_Size", row.get("Grid_Size_X", "")), row["Dispatch_Id"])
    per[key][row["Counter_Name"]] += float(row["Counter_Value"])
agg = collections.defaultdict(list)
for (name, grid, _), c in per.items():
    agg[(name, grid)].append(c)
for (name, grid), lst in agg.items():
    c = {k: sum(x[k] for x in lst) / len(lst) for k in lst[0]}
    cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8
    busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(cyc * 256 * 4, 1)
    wc = max(c.get("SQ_WAVE_CYCLES", 0), 1)
    if len(sys.argv) > 2:  # raw per-dispatch averages
        print(f"{name} grid={grid} n={len(lst)} " + " ".join(f"{k}={v:.4g}" for k, v in sorted(c.items())))
        continue
    print(f"{name} grid={grid} n={len(lst)} cycles={cyc:.0f} mfma_busy={busy:.3f} "
          f"wait_inst={c.get('SQ_WAIT_INST_ANY', 0) / wc:.3f} wait_any={c.get('SQ_WAIT_ANY', 0) / wc:.3f} "
          f"active={c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.3f}")
