"""A/B of the batched cornerSubPix variants (COEB_SUBPIX_VARIANT) inside the device Frame ctor of
a 257-frame batch: run under rocprofv3 --kernel-trace --stats once per variant; prints the
iteration count per corner (COEB_SUBPIX_COUNT).  Usage: python tools/subpix_ab.py [--steps N]"""
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
    cnt = np.zeros(2, np.int32)
    bp.run(rgbd=True, frame=True, match=False)
    bp.synchronize()
    L.coeb_internal_subpix_count(cnt.ctypes.data)
    for _ in range(args.steps):
        bp.run(rgbd=True, frame=True, match=False)
    bp.synchronize()
    L.coeb_internal_subpix_count(cnt.ctypes.data)
    tms, _ = bp.ctx.batch_frame_results(F, F)
    clk = np.zeros(8, np.uint64)
    L.coeb_internal_subpix_clock.argtypes = [C.c_void_p]
    L.coeb_internal_subpix_clock(clk.ctypes.data)       # zeros unless built with COEB_SUBPIX_CLOCK
    if clk[4]:
        n = float(clk[4])
        print(json.dumps(dict(per_iteration_cycles=dict(fill=round(clk[0] / n), terms=round(clk[1] / n),
                                                        sums=round(clk[2] / n)),
                              per_corner_cycles=round(float(clk[3]) / max(1, cnt[1])))))
    print(json.dumps(dict(variant=os.environ.get("COEB_SUBPIX_VARIANT", "1"), iterations=int(cnt[0]),
                          corners=int(cnt[1]), iters_per_corner=round(float(cnt[0]) / max(1, cnt[1]), 3),
                          tm_points=int(sum(len(t) for t in tms if t is not None)))))
    bp.close()


if __name__ == "__main__":
    main()
