"""k_fast_band phase clocks (library built with -DCOEB_BAND_CLOCK=1, loaded through
COEB_LIB_PATH): wave 0's clock64 cycles per phase summed over all workgroups of one
257-frame config-A extraction.  Diagnostic only."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "coeb-slam_amd"))
from coeb_front import synth  # noqa: E402
from coeb_front.pipeline import BatchPipeline  # noqa: E402

F = 257
fr = synth.make_frames(640, 480, F, seed=1)
bp = BatchPipeline(640, 480, F)
bp.load(fr, Tcw=np.stack([synth.motion_pose()] * F))
bp.run(match=False)
bp.synchronize()
bp.ctx.debug_read("band_timing")          # clears
for _ in range(3):
    bp.run(match=False)
bp.synchronize()
t = bp.ctx.debug_read("band_timing").view(np.uint64).astype(np.float64) / 3
names = ["stage", "phase2+barrier", "nms", "keep", "output", "w0 flushes", "w0 phase2"]
tot = t[[0, 1, 2, 3, 4]].sum()
for i, n in enumerate(names):
    print("%-16s %14.0f cycles  %5.1f %%" % (n, t[i], 100 * t[i] / tot))
