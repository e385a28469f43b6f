"""Iteration counts of the batched ProcessMovingObject stages inside the device Frame ctor of a
config-D batch (COEB_SUBPIX_COUNT builds them in: cornerSubPix iterations per corner, LK
iterations per point summed over the pyramid levels).  Run it under rocprofv3 --kernel-trace
--stats for the per-kernel times.  Usage: python tools/flow_counts.py [--steps N] [--frames F]"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "coeb-slam_amd"))
sys.path.insert(0, ROOT)
os.environ.setdefault("COEB_SUBPIX_COUNT", "1")
os.environ["COEB_EXPERIMENTS"] = "1"     # experiment switches are read only under this gate


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--frames", type=int, default=257)
    args = ap.parse_args()
    import bench
    import coeb_front as cf
    from coeb_front.pipeline import BatchPipeline
    F = args.frames
    bp = BatchPipeline(640, 480, F)
    bench.load_batch(bp, bench.CONFIGS["D"], 640, 480, F, 0)
    L = cf.lib()
    L.coeb_internal_subpix_count.argtypes = [C.c_void_p]
    cnt = np.zeros(4, np.int32)
    bp.run(rgbd=True, frame=True, match=False)
    bp.synchronize()
    L.coeb_internal_subpix_count(cnt.ctypes.data)          # clears
    for _ in range(args.steps):
        bp.run(rgbd=True, frame=True, match=False)
    bp.synchronize()
    L.coeb_internal_subpix_count(cnt.ctypes.data)
    print(json.dumps(dict(subpix_iterations=int(cnt[0]), corners=int(cnt[1]),
                          subpix_iters_per_corner=round(float(cnt[0]) / max(1, cnt[1]), 3),
                          lk_iterations=int(cnt[2]), lk_points=int(cnt[3]),
                          lk_iters_per_point=round(float(cnt[2]) / max(1, cnt[3]), 3))))
    bp.close()


if __name__ == "__main__":
    main()
