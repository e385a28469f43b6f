#!/usr/bin/env python3
"""Per-dispatch summary of a rocprofv3 --kernel-trace CSV: average duration per (kernel, grid),
so the launches of one kernel at different sizes (k_pyr_level per pyramid level, k_fast /
k_blur split over streams) are told apart.  Usage: ktrace_summary.py run_kernel_trace.csv"""
import csv
import sys
from collections import defaultdict


def main(path):
    rows = list(csv.DictReader(open(path)))
    agg = defaultdict(list)
    for r in rows:
        kn = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        name = kn.split("(")[0].split("<")[0].strip()
        grid = (int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0), int(r.get("Grid_Size_Y", 0) or 0),
                int(r.get("Grid_Size_Z", 0) or 0))
        agg[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    print("%-28s %-22s %6s %10s %10s" % ("kernel", "grid", "n", "avg_us", "total_us"))
    for (name, grid), d in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print("%-28s %-22s %6d %10.1f %10.1f" % (name, "x".join(map(str, grid)), len(d), sum(d) / len(d), sum(d)))


if __name__ == "__main__":
    main(sys.argv[1])
