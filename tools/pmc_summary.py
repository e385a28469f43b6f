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


# FETCH_SIZE scale, calibrated on this chip (tools/micro/fetch_calib.hip, profiles/r05/s1/calib.log):
# a 1.2 GB buffer (past the 256 MiB Infinity Cache) read exactly once in each of the product kernels'
# load shapes -- 16 B per lane streaming, 4 B per lane streaming, k_fast's lane-per-row 3 x 16 B
# windows (register staging), k_fast's byte-granular 48-B LDS-DMA rows, k_describe's 37 x 64 B patch
# rows -- reports FETCH_SIZE = 0.500 x the bytes in every shape (the DMA rows: 0.500 x the whole
# 64-B lines they touch).  So FETCH_SIZE counts half of every line the L2 requests, whatever the
# access width: one scale of 2 for all kernels (the round-4 summary kept 1 for the <= 4-B-load
# kernels, from k_blur's fetches matching its byte count; the calibration says those were 2x too).
FETCH_SCALE = 2.0


def traffic_json(merged, nd, frames, command, fetch_scale=FETCH_SCALE):
    """Per kernel, memory-side bytes per launch: fetch_scale x FETCH_SIZE + WRITE_SIZE (rocprofv3
    KB).  FETCH_SIZE counts L2 requests to the fabric, Infinity-Cache hits included
    (MI355X_MICROARCH.md HBM), so this is the traffic past L2, an upper bound on HBM bytes."""
    out = dict(frames_per_launch=frames, command=command, fetch_scale=fetch_scale,
               calibration="tools/micro/fetch_calib.hip: FETCH_SIZE = 0.500 x the bytes of every load shape "
                           "(profiles/r05/s1/calib.log)",
               correction="bytes = (%g * FETCH_SIZE + WRITE_SIZE) * 1024 per dispatch, mean over dispatches"
                          % fetch_scale,
               kernels={})
    for k, cv in sorted(merged.items()):
        if "FETCH_SIZE" not in cv or "WRITE_SIZE" not in cv:
            continue
        sc = fetch_scale
        out["kernels"][k] = dict(fetch_kb=round(cv["FETCH_SIZE"], 3), write_kb=round(cv["WRITE_SIZE"], 3),
                                 fetch_scale=sc, traffic_bytes=int((sc * cv["FETCH_SIZE"] + cv["WRITE_SIZE"]) * 1024),
                                 dispatches=nd[k])
    return out


VALU_PER_CU_CYCLE = 2.0   # MI355X_MICROARCH.md: 4 SIMD-32 per CU, a wave64 VALU op issues over 2 cycles


def valu_json(merged, nd, frames, command, n_cu=256, n_xcd=8, rate=VALU_PER_CU_CYCLE):
    """Per kernel, VALU wave-instructions per launch and the fraction of the chip's VALU issue
    rate they fill: a CU issues at most two wave64 VALU instructions per cycle (4 SIMD-32 units,
    each taking 2 cycles per wave64 instruction), and GRBM_GUI_ACTIVE sums the busy cycles of
    the 8 XCDs."""
    out = dict(frames_per_launch=frames, command=command,
               definition="valu_issue_frac = SQ_INSTS_VALU / (%g x %d CUs x GRBM_GUI_ACTIVE / %d XCDs), per dispatch "
                          "(%g wave64 VALU instructions per CU per cycle)" % (rate, n_cu, n_xcd, rate), kernels={})
    for k, cv in sorted(merged.items()):
        if "SQ_INSTS_VALU" not in cv or not cv.get("GRBM_GUI_ACTIVE"):
            continue
        cycles = cv["GRBM_GUI_ACTIVE"] / n_xcd
        e = out["kernels"][k] = dict(valu_insts=int(cv["SQ_INSTS_VALU"]), busy_cycles=int(cycles),
                                     valu_issue_frac=round(cv["SQ_INSTS_VALU"] / (rate * n_cu * cycles), 4),
                                     dispatches=nd[k])
        # stall fractions of the resident wave-cycles and LDS bank conflicts per LDS instruction
        if cv.get("SQ_WAVE_CYCLES"):
            for key, cnt in (("wait_inst_frac", "SQ_WAIT_INST_ANY"), ("wait_any_frac", "SQ_WAIT_ANY"),
                             ("active_inst_frac", "SQ_ACTIVE_INST_ANY")):
                if cnt in cv:
                    e[key] = round(cv[cnt] / cv["SQ_WAVE_CYCLES"], 4)
        if cv.get("SQ_INSTS_LDS") and "SQ_LDS_BANK_CONFLICT" in cv:
            e["lds_conflict_per_lds_inst"] = round(cv["SQ_LDS_BANK_CONFLICT"] / cv["SQ_INSTS_LDS"], 3)
    return out


if __name__ == "__main__":
    import argparse
    import json
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--json", help="write per-kernel HBM traffic per launch (for bench.py roofline.traffic)")
    ap.add_argument("--frames", type=int, default=0, help="frames per launch of the profiled command")
    ap.add_argument("--command", default="")
    ap.add_argument("--size", default="640x480", help="frame size of the profiled command (WxH)")
    ap.add_argument("--fetch-scale", type=float, default=FETCH_SCALE)
    ap.add_argument("--valu-json", help="write per-kernel VALU issue utilisation (SQ_INSTS_VALU, GRBM_GUI_ACTIVE)")
    a = ap.parse_args()
    merged = collections.defaultdict(dict)
    nd = {}
    for p in a.csv:
        for k, (cv, n, g) in load(p).items():
            merged[k].update(cv)
            nd[k] = n
    for k, cv in sorted(merged.items()):
        print("%-16s n=%-3d %s" % (k, nd[k], " ".join("%s=%.4g" % (c, v) for c, v in sorted(cv.items()))))
    wh = dict(zip(("width", "height"), map(int, a.size.split("x"))))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(dict(wh, **traffic_json(merged, nd, a.frames, a.command, a.fetch_scale)), f, indent=1)
    if a.valu_json:
        with open(a.valu_json, "w") as f:
            json.dump(dict(wh, **valu_json(merged, nd, a.frames, a.command)), f, indent=1)
