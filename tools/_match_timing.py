"""k_match phase clocks over one bench-shaped batch (COEB_MATCH_TIMING=1): median cycles per
phase across the batch's pairs.  Diagnostic only.  Optional arguments: W H F NFEATURES
(default 640 480 257 1000; 1280 960 33 2000 is one pipeline of config B's 64-frame shard)."""
import os
import sys

import numpy as np

os.environ["COEB_MATCH_TIMING"] = "1"
os.environ["COEB_EXPERIMENTS"] = "1"     # experiment switches are read only under this gate
# (and the library must be an experiment build: tools/_build_var.sh clock "-DCOEB_MATCH_CLOCK=1")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "coeb-slam_amd"))
from coeb_front import synth  # noqa: E402
from coeb_front.pipeline import BatchPipeline  # noqa: E402

W, H, F, NF = (int(a) for a in sys.argv[1:5]) if len(sys.argv) > 4 else (640, 480, 257, 1000)
fr = synth.make_frames(W, H, F, seed=1)
bp = BatchPipeline(W, H, F, nfeatures=NF)
bp.load(fr, Tcw=np.stack([synth.motion_pose()] * F))
for _ in range(3):
    bp.run()
bp.ctx.synchronize()
t = bp.ctx.debug_read("match_timing").view(np.int64).reshape(-1, 16)[:F - 1]
names = ["grid", "lists0", "claims0", "gap0", "assign0", "lists1", "claims1", "gap1", "assign1"]
d = np.stack([t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2], t[:, 4] - t[:, 3], t[:, 5] - t[:, 4],
              np.where(t[:, 6] > 0, t[:, 6] - t[:, 5], 0), np.where(t[:, 7] > 0, t[:, 7] - t[:, 6], 0),
              np.where(t[:, 8] > 0, t[:, 8] - t[:, 7], 0), np.where(t[:, 9] > 0, t[:, 9] - t[:, 8], 0)], 1)
tot = t[:, 10] - t[:, 0]
print("total cycles median %d max %d" % (np.median(tot), tot.max()))
for i, nme in enumerate(names):
    print("%-8s median %8d  max %8d" % (nme, np.median(d[:, i]), d[:, i].max()))
print("fixpoint iterations attempt0 median %d max %d; retried pairs %d" % (np.median(t[:, 12]), t[:, 12].max(),
                                                                         int((t[:, 6] > 0).sum())))
print("lists phase per-wave loop time: slowest %d, fastest %d cycles (median over pairs), %d passes" %
      (np.median(t[:, 13]), np.median(t[:, 14]), np.median(t[:, 15])))
