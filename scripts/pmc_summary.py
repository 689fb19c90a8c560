"""Summarise rocprofv3 PMC passes into profiles/pmc_traffic.json (bench.py roofline.traffic).

    python scripts/pmc_summary.py ROUND [OUT] [--workload variant=large_v3,weights=q4_0,precision=f16x2,clips=32]
        (reads gpurun_out/pmc_{FETCH_SIZE,WRITE_SIZE}_ROUND, writes OUT, default
        profiles/pmc_traffic.json)

The workload the passes profiled is recorded in the summary; bench.py uses a
summary only for a run of the same variant, weights, precision and clips.

HBM bytes per launch = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes): on gfx950
FETCH_SIZE reports half the bytes of a 16-B-per-lane streaming read and
WRITE_SIZE the exact bytes of 16-B / dword stores (MI355X_MICROARCH.md, HBM).
The doubling is calibrated for 16-B-per-lane reads only; the undoubled
figure (FETCH_SIZE + WRITE_SIZE) is reported beside it for kernels whose
reads are narrower.
"""
import csv
import glob
import json
import os
import re
import sys

FAMILIES = {"q4_gemm_prefill_kernel": r"q4_gemm_prefill_kernel", "q4_gemm_wide_kernel": r"q4_gemm_wide_kernel",
            "q4_gemm_decode_kernel": r"q4_gemm_decode_kernel",
            "xattn_main_kernel": r"xattn_main_kernel",
            "xattn_q_kernel": r"xattn_q_\w*kernel", "xattn_merge_kernel": r"xattn_merge_kernel",
            "xattn_out_kernel": r"xattn_out_kernel"}


def grid_items(row: dict) -> int:
    """Total work-items of the dispatch (Grid_Size, or the product of Grid_Size_X/Y/Z)."""
    if row.get("Grid_Size"):
        return int(float(row["Grid_Size"]))
    n = 1
    for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"):
        if row.get(k):
            n *= int(float(row[k]))
    return n


def load(counter: str, rnd: str, by_grid: dict | None = None) -> dict:
    files = glob.glob(f"gpurun_out/pmc_{counter}_{rnd}/**/*counter_collection*.csv", recursive=True)
    per = {}
    for fn in files:
        for row in csv.DictReader(open(fn)):
            name, cname = row.get("Kernel_Name", ""), row.get("Counter_Name", "")
            if cname != counter:
                continue
            for fam, rx in FAMILIES.items():
                if re.search(rx, name):
                    per.setdefault(fam, []).append(float(row["Counter_Value"]))
                    if by_grid is not None:
                        by_grid.setdefault((fam, grid_items(row)), []).append(float(row["Counter_Value"]))
    return per


DEFAULT_WORKLOAD = {"variant": "large_v3", "weights": "q4_0", "precision": "f16x2", "clips": 32}


def parse_workload(argv: list[str]) -> dict:
    w = dict(DEFAULT_WORKLOAD)
    if "--workload" in argv:
        for kv in argv[argv.index("--workload") + 1].split(","):
            k, v = kv.split("=", 1)
            w[k] = int(v) if k == "clips" else v
    return w


def main() -> None:
    argv = [a for a in sys.argv[1:]]
    workload = parse_workload(argv)
    if "--workload" in argv:
        i = argv.index("--workload")
        del argv[i: i + 2]
    rnd = argv[0] if argv else "r01"
    gf, gw = {}, {}
    fetch, write = load("FETCH_SIZE", rnd, gf), load("WRITE_SIZE", rnd, gw)
    out = {"round": rnd, "workload": workload, "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes; "
                                   "hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 per launch",
           "kernels": {}}
    for fam in FAMILIES:
        f, w = fetch.get(fam, []), write.get(fam, [])
        if not f or not w:
            continue
        fk, wk = sum(f) / len(f), sum(w) / len(w)
        out["kernels"][fam] = {"launches_fetch": len(f), "launches_write": len(w), "fetch_size_kib": fk,
                               "write_size_kib": wk, "hbm_bytes_per_launch": (2 * fk + wk) * 1024,
                               "hbm_bytes_per_launch_undoubled": (fk + wk) * 1024}
        # the same family split by dispatch size (work-items): decode groups,
        # prompts and the bench's all-clip probe launch differ only in grid
        grids = {}
        for (fam2, g), fv in sorted(gf.items()):
            wv = gw.get((fam2, g), [])
            if fam2 != fam or not wv:
                continue
            a, b = sum(fv) / len(fv), sum(wv) / len(wv)
            grids[str(g)] = {"launches": len(fv), "hbm_bytes_per_launch": (2 * a + b) * 1024,
                             "hbm_bytes_per_launch_undoubled": (a + b) * 1024}
        out["kernels"][fam]["by_grid_items"] = grids
    dst = argv[1] if len(argv) > 1 else "profiles/pmc_traffic.json"
    os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
