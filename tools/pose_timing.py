#!/usr/bin/env python3
"""Per-call time of coeb_pose_optimization against the edge count (fixed serial cost vs
per-edge cost of k_pose).  Diagnostic only: python tools/pose_timing.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "coeb-slam_amd"))
import numpy as np  # noqa: E402
import coeb_front as cf  # noqa: E402
from coeb_front import synth  # noqa: E402


def main():
    ctx = cf.Context(max_width=640, max_height=480, max_batch=4)
    cam = cf.make_camera(synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF, 640, 480)
    out = {}
    for n in (20, 100, 250, 500, 1000):
        P = synth.make_pose_problem(n=n, seed=1)

        def once():
            Fp = cf.Frame(P["kps"], np.zeros((len(P["kps"]), 32), np.uint8), P["ur"], Tcw=P["Tcw_init"])
            Fp.mvpMapPoints = np.where(P["has_mp"] > 0, 0, -1).astype(np.int32)
            Fp.mvMapPointPos = P["xw"]
            return cf.Optimizer.PoseOptimization(Fp, cam, ctx)
        once()
        t0 = time.perf_counter()
        for _ in range(10):
            r = once()
        out[n] = dict(ms=round((time.perf_counter() - t0) / 10 * 1e3, 4), edges=int(P["has_mp"].sum()), inliers=int(r))
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
