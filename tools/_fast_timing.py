"""Per-cell k_fast phase clocks (library built with -DCOEB_FAST_CLOCK=1, loaded through
COEB_LIB_PATH; run with COEB_SIDE_STREAM=0): lane 0's clock64 cycles per phase summed over all
cells of one 257-frame config-A extraction, and per cell.  Diagnostic only."""
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
bp.ctx.debug_read("fast_timing")          # clears
for _ in range(3):
    bp.run(match=False)
bp.synchronize()
t = bp.ctx.debug_read("fast_timing").view(np.uint64).astype(np.float64) / 3
cells = max(t[5], 1)
names = ["wait+stage+clear", "pre-test passes", "strength flushes", "nms+output", "total (wave)"]
for i, n in enumerate(names):
    print("%-18s %14.0f cycles  %8.0f per cell  %5.1f %% of total" % (n, t[i], t[i] / cells, 100 * t[i] / t[4]))
print("cells %.0f  corners per cell %.1f" % (cells, t[6] / cells))
