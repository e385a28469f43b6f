"""k_pose phase clocks over one config-D batch (COEB_POSE_TIMING=1): median clock64 cycles
per phase across the 256 frames.  Diagnostic only; needs a library built with the clocks compiled in:
tools/_build_var.sh clock "-DCOEB_POSE_CLOCK=1" and COEB_LIB_PATH=coeb-slam_amd/lib/var_clock.so."""
import os
import sys

import numpy as np

os.environ["COEB_POSE_TIMING"] = "1"
os.environ["COEB_EXPERIMENTS"] = "1"     # experiment switches are read only under this gate
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "coeb-slam_amd"))
from coeb_front import synth  # noqa: E402
from coeb_front.pipeline import BatchPipeline  # noqa: E402

F = 257
fr = synth.make_frames(640, 480, F, seed=1)
bp = BatchPipeline(640, 480, F)
bp.load(fr, Tcw=np.stack([synth.motion_pose()] * F))
bp.run(pose=True)
bp.ctx.synchronize()
t = bp.ctx.debug_read("pose_timing").view(np.int64).reshape(-1, 8)[1:F]
names = ["chi2 passes", "build passes", "thread-0 solve/exp", "classification", "total"]
for i, nme in enumerate(names):
    print("%-20s median %10d  max %10d" % (nme, np.median(t[:, i]), t[:, i].max()))
print("iterations median %d, trials median %d" % (np.median(t[:, 5]), np.median(t[:, 6])))
