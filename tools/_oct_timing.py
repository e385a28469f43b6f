"""k_octree per-workgroup clocks over one extraction (default 257 frames of config A; args W H F) (library built with
-DCOEB_OCT_CLOCK=1, loaded through COEB_LIB_PATH; COEB_SIDE_STREAM=0).  Diagnostic only."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "coeb-slam_amd"))
from coeb_front import synth  # noqa: E402
from coeb_front.pipeline import BatchPipeline  # noqa: E402

W, H, F = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (640, 480, 257)))
NF = 2000 if W >= 1280 else 1000
fr = synth.make_frames(W, H, F, seed=1)
bp = BatchPipeline(W, H, F, nfeatures=NF)
bp.load(fr, Tcw=np.stack([synth.motion_pose()] * F))
for _ in range(3):
    bp.run(match=False)
bp.synchronize()
t = bp.ctx.debug_read("oct_timing").view(np.int64).reshape(4096, 6)[:F * 8]
w0 = t[:, 2].min()
for l in range(8):
    r = t[t[:, 0] == l]
    print("level %d: WGs %d  K median %d max %d  cycles median %d max %d  (gather+init %d, main loop %d)  start %.1f..%.1f us"
          % (l, len(r), np.median(r[:, 1]), r[:, 1].max(), np.median(r[:, 3]), r[:, 3].max(), np.median(r[:, 4]),
             np.median(r[:, 5]), (r[:, 2].min() - w0) / 100.0, (r[:, 2].max() - w0) / 100.0))
