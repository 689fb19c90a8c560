"""profiles/xattn_in_graph.json from a chain trace's per-grid table
(scripts/trace_by_grid.py output) + the bench workload it ran:
    python3 scripts/in_graph_summary.py <chain_grid.json> <variant> <weights> <precision> <clips> <out.json>"""
import json
import sys

grid, variant, weights, prec, clips, out = sys.argv[1:7]
rows = [e for e in json.load(open(grid)) if e["kernel"].startswith("xattn")]
json.dump({"workload": {"variant": variant, "weights": weights, "precision": prec, "clips": int(clips)},
           "source": "rocprofv3 --kernel-trace of bench.py (scripts/gpu.sh trace), decode graphs replayed",
           "kernels": rows}, open(out, "w"), indent=1)
