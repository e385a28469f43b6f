#!/usr/bin/env python3
"""The drop-in single-frame path alone (bench.single_frame_timing: coeb_extract +
coeb_stereo_from_rgbd + coeb_match_lastframe per frame, frame i against frame i-1), for a
rocprofv3 kernel / memory-copy trace of exactly those calls (tools/single_frame_trace.py reads it)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "coeb-slam_amd"))
import bench  # noqa: E402

if __name__ == "__main__":
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    print(json.dumps(bench.single_frame_timing(640, 480, reps=reps)), flush=True)
