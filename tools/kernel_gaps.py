"""Bench-only: per-kernel mean duration and mean gap to the next dispatch from a
rocprofv3 kernel trace (`--kernel-trace --output-format csv`, the *_kernel_trace.csv file).

Dispatches are grouped by (kernel name, grid size); the gap of a dispatch is the next
dispatch's start minus its end on the same queue, when the next one is the same group
(back-to-back launches of one shape, as tools/small_n_probe.py issues them).

Usage: python tools/kernel_gaps.py TRACE.csv [--min-count 50]
"""
import argparse
import csv
import json
import statistics
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--min-count", type=int, default=50)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    key_q = "Queue_Id" if rows and "Queue_Id" in rows[0] else None
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    by_q = {}
    for r in rows:
        by_q.setdefault(r.get(key_q, "0") if key_q else "0", []).append(r)
    stats = {}
    for q, rs in by_q.items():
        for i, r in enumerate(rs):
            grid = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
            k = (r["Kernel_Name"][:90], grid)
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            s = stats.setdefault(k, {"dur": [], "gap": []})
            s["dur"].append(d)
            if i + 1 < len(rs):
                nx = rs[i + 1]
                if (nx["Kernel_Name"][:90], nx.get("Grid_Size_X") or nx.get("Grid_Size") or "?") == k:
                    s["gap"].append((int(nx["Start_Timestamp"]) - int(r["End_Timestamp"])) / 1e3)
    out = []
    for (name, grid), s in stats.items():
        if len(s["dur"]) < a.min_count:
            continue
        out.append({"kernel": name, "grid": grid, "count": len(s["dur"]),
                    "mean_us": round(statistics.mean(s["dur"]), 3),
                    "median_us": round(statistics.median(s["dur"]), 3),
                    "gap_median_us": round(statistics.median(s["gap"]), 3) if s["gap"] else None})
    out.sort(key=lambda r: (r["kernel"], int(r["grid"]) if str(r["grid"]).isdigit() else 0))
    for r in out:
        print(json.dumps(r))
    return 0


if __name__ == "__main__":
    sys.exit(main())
