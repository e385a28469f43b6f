"""Per-call timing of Frame::ProcessMovingObject on the device (host-buffer entry and the
device-resident entry), for rocprofv3 kernel traces of the k_gf_* / k_subpix / k_lk / k_fm
kernels.  Usage: python tools/flow_bench.py [--calls N]"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "coeb-slam_amd"))
import coeb_front as cf  # noqa: E402
from coeb_front import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=50)
    args = ap.parse_args()
    prev, cur, _ = synth.moving_object_pair(640, 480, 0)
    ctx = cf.Context(max_width=640, max_height=480, max_batch=2)
    L = cf.lib()
    tm = np.zeros((1024, 2), np.float32)
    nt = C.c_int(0)
    for _ in range(3):
        cf.ProcessMovingObject(ctx, prev, cur)
    t0 = time.perf_counter()
    for _ in range(args.calls):
        cf.ProcessMovingObject(ctx, prev, cur)
    host_ms = (time.perf_counter() - t0) / args.calls * 1e3
    buf = C.c_void_p()
    ctx.check(L.coeb_device_alloc(ctx.h, 2 * prev.size, C.byref(buf)))
    ctx.check(L.coeb_memcpy_h2d(ctx.h, buf, prev.ctypes.data, prev.size))
    ctx.check(L.coeb_memcpy_h2d(ctx.h, C.c_void_p(buf.value + prev.size), cur.ctypes.data, cur.size))
    dev = lambda: ctx.check(L.coeb_moving_object_points_device(ctx.h, buf, C.c_void_p(buf.value + prev.size), 640, 480,
                                                                640, cf._p(tm), len(tm), C.byref(nt), None))
    dev()
    t0 = time.perf_counter()
    for _ in range(args.calls):
        dev()
    dev_ms = (time.perf_counter() - t0) / args.calls * 1e3
    L.coeb_device_free(ctx.h, buf)
    print(json.dumps({"process_moving_object": {"host_entry_ms": round(host_ms, 4), "device_entry_ms": round(dev_ms, 4),
                                                "n_tm": nt.value, "calls": args.calls}}))
    ctx.close()


if __name__ == "__main__":
    main()
