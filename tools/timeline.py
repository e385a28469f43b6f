"""Kernel timeline of the last extraction step in a rocprofv3 kernel trace (csv): launches from
the last k_dynmask on, start / end in microseconds from that k_dynmask's start, per queue."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows = [r for r in rows if not r["Kernel_Name"].startswith("__amd")]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_dynmask" in r["Kernel_Name"]]
i0 = starts[-2] if len(starts) > 1 else starts[-1]
i1 = starts[-1]
t0 = int(rows[i0]["Start_Timestamp"])
step = rows[i0:i1]
end = max(int(r["End_Timestamp"]) for r in step)
print("step (dynmask to last end): %.1f us" % ((end - t0) / 1000))
for r in step:
    name = r["Kernel_Name"].split("(")[0].replace("(anonymous namespace)::", "").replace("void ", "")
    s, e = (int(r["Start_Timestamp"]) - t0) / 1000, (int(r["End_Timestamp"]) - t0) / 1000
    print("%-22s q%-3s %8.1f %8.1f %7.1f  grid %s x %s x %s" % (name[:22], r["Queue_Id"], s, e, e - s,
          r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"]))
