#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs per kernel (mean per dispatch).  FETCH_SIZE / WRITE_SIZE are
in KB; on gfx950 FETCH_SIZE under-counts wide streaming reads by 2x (MI355X_MICROARCH.md HBM)."""
import collections
import csv
import re
import sys


def load(path):
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    grid = {}
    for r in rows:
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        k = m.group(1) if m else r["Kernel_Name"][:24]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
        grid[k] = r["Grid_Size"]
    return {k: ({c: v / len(disp[k]) for c, v in agg[k].items()}, len(disp[k]), grid[k]) for k in agg}


if __name__ == "__main__":
    merged = collections.defaultdict(dict)
    nd = {}
    for p in sys.argv[1:]:
        for k, (cv, n, g) in load(p).items():
            merged[k].update(cv)
            nd[k] = n
    for k, cv in sorted(merged.items()):
        print("%-16s n=%-3d %s" % (k, nd[k], " ".join("%s=%.4g" % (c, v) for c, v in sorted(cv.items()))))
