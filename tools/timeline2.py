#!/usr/bin/env python3
"""Kernel timeline of one whole bench step in a rocprofv3 kernel trace (csv), for P pipelines per
step (P k_dynmask launches per step): launches from the P-th last-but-one group of k_dynmask on,
start / end in us from the first of them, per queue; then the union of busy time (any kernel
running) and, per kernel, the time it ran with no other kernel beside it.
Usage: timeline2.py run_kernel_trace.csv [pipelines=2]"""
import csv
import sys


def main(path, P=2):
    rows = [r for r in csv.DictReader(open(path)) if not r["Kernel_Name"].startswith("__amd")]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "k_dynmask" in r["Kernel_Name"]]
    if len(starts) < 2 * P:
        print("need >= %d k_dynmask launches" % (2 * P))
        return
    i0, i1 = starts[-2 * P], starts[-P]
    t0 = int(rows[i0]["Start_Timestamp"])
    step = rows[i0:i1]
    iv = []
    for r in step:
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        name = name.split("<")[0].strip()
        s, e = (int(r["Start_Timestamp"]) - t0) / 1000, (int(r["End_Timestamp"]) - t0) / 1000
        iv.append((s, e, name, r["Queue_Id"]))
        print("%-16s q%-3s %8.1f %8.1f %7.1f  grid %s x %s x %s" % (name[:16], r["Queue_Id"], s, e, e - s,
              r.get("Grid_Size_X", "?"), r.get("Grid_Size_Y", "?"), r.get("Grid_Size_Z", "?")))
    next_start = (int(rows[i1]["Start_Timestamp"]) - t0) / 1000
    # union of busy intervals and solo time per kernel
    ev = sorted(set([x for s, e, _, _ in iv for x in (s, e)]))
    busy = 0.0
    solo = {}
    for a, b in zip(ev, ev[1:]):
        run = [n for s, e, n, _ in iv if s <= a and e >= b]
        if run:
            busy += b - a
        if len(run) == 1:
            solo[run[0]] = solo.get(run[0], 0.0) + (b - a)
    print("step %.1f us (first k_dynmask to the next step's), busy %.1f us, idle %.1f us" %
          (next_start, busy, next_start - busy))
    tot = {}
    for s, e, n, _ in iv:
        tot[n] = tot.get(n, 0.0) + (e - s)
    print("%-16s %10s %10s" % ("kernel", "sum_us", "solo_us"))
    for n, t in sorted(tot.items(), key=lambda kv: -kv[1]):
        print("%-16s %10.1f %10.1f" % (n, t, solo.get(n, 0.0)))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2)
