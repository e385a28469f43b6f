#!/usr/bin/env python3
"""Device timeline of the last frames of a rocprofv3 --kernel-trace --memory-copy-trace run of
tools/single_frame.py: every kernel and copy with its duration and the idle gap before it, then
per-frame totals (a frame starts at k_dynmask, the first kernel of coeb_extract).
Usage: sf_timeline.py <trace dir> [frames]"""
import csv
import glob
import os
import sys


def main(d, nfr=4):
    ev = []
    for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            kn = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].split("<")[0]
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + kn.strip()))
    for p in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C " + r["Direction"].replace("MEMORY_COPY_", "")))
    ev.sort()
    starts = [i for i, e in enumerate(ev) if e[2] == "K k_dynmask"]
    if len(starts) < nfr + 2:
        print("too few frames (%d)" % len(starts))
        return
    spans, busys, kern = [], [], []
    for a, b in zip(starts[-nfr - 1:-1], starts[-nfr:]):
        fr = ev[a:b]
        t0 = fr[0][0]
        prev = t0
        busy = 0
        print("---- frame")
        for s, e, k in fr:
            print("%8.1f %7.1f gap %6.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, (s - prev) / 1e3, k))
            busy += max(0, e - max(s, prev))
            prev = max(prev, e)
        spans.append((ev[b][0] - t0) / 1e3)
        busys.append(busy / 1e3)
        kern.append(sum(e - s for s, e, k in fr if k[0] == "K") / 1e3)
    m = lambda x: sum(x) / len(x)
    print("per frame (frame start to next frame start): %.1f us, device busy %.1f us (kernels %.1f), idle %.1f us"
          % (m(spans), m(busys), m(kern), m(spans) - m(busys)))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 4)
