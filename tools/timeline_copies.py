"""Print a rocprofv3 kernel + memory-copy timeline (ms from the first record) from a
--kernel-trace --memory-copy-trace CSV output prefix: one line per copy and per kernel run
(consecutive kernels on one queue merged), to see what a pipeline step waits for."""
import csv
import sys

pre = sys.argv[1]
ev = []
for r in csv.DictReader(open(pre + "_kernel_trace.csv")):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K q%s" % r.get("Queue_Id", "?"),
               r["Kernel_Name"].split("(")[0].replace("(anonymous namespace)::", "")[-28:]))
for r in csv.DictReader(open(pre + "_memory_copy_trace.csv")):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY", "%s %s B" % (r.get("Direction", r.get("Kind", "")), r.get("Size", ""))))
ev.sort()
t0 = ev[0][0]
merged = []
for s, e, kind, name in ev:
    if merged and kind.startswith("K") and merged[-1][2] == kind and s - merged[-1][1] < 20000:
        merged[-1][1] = max(merged[-1][1], e)
        merged[-1][4] += 1
        continue
    merged.append([s, e, kind, name, 1])
for s, e, kind, name, n in merged:
    if kind == "COPY" or e - s > 50000:
        print("%9.3f %9.3f %7.3f  %-6s %s%s" % ((s - t0) / 1e6, (e - t0) / 1e6, (e - s) / 1e6, kind, name, "" if n == 1 else " (+%d kernels)" % (n - 1)))
