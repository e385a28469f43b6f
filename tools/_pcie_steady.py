"""Diagnostic: HostStream batch completion times (host clock) for N config-A batches submitted
back to back, to separate the pipeline's steady-state interval from its fill / drain."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "coeb-slam_amd"))
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
from coeb_front import HostBuffer, synth  # noqa: E402
from coeb_front.pipeline import HostStream  # noqa: E402

F, W, H = 257, 640, 480
N = int(sys.argv[1]) if len(sys.argv) > 1 else 40
fr = synth.make_frames(W, H, F, seed=1)
hs = HostStream(W, H, F, Tcw=np.stack([synth.motion_pose()] * F))
src = HostBuffer(F * H * W)
src.view(np.uint8, (F, H, W))[:] = fr
for i in range(4):
    hs.submit(i, src)
hs.wait(2)
hs.wait(3)
t0 = time.perf_counter()
sub = []
for i in range(4, 4 + N):
    hs.submit(i, src)
    sub.append(time.perf_counter() - t0)
done = []
for i in range(4, 4 + N):
    hs.wait(i)
    done.append(time.perf_counter() - t0)
sub, done = np.array(sub) * 1e3, np.array(done) * 1e3
print("submit times (ms): first %.2f last %.2f, per batch %.3f" % (sub[0], sub[-1], (sub[-1] - sub[0]) / (N - 1)))
print("completion (ms): first %.2f last %.2f" % (done[0], done[-1]))
d = np.diff(done)
print("completion intervals: median %.3f mean %.3f min %.3f max %.3f" % (np.median(d), d.mean(), d.min(), d.max()))
print("steady state (batches %d..%d): %.3f ms per batch = %.0f frames/s" %
      (N // 4, N - 1, (done[-1] - done[N // 4]) / (N - 1 - N // 4), (F - 1) / ((done[-1] - done[N // 4]) / (N - 1 - N // 4)) * 1e3))
print("whole run incl. fill and drain: %.3f ms per batch" % (done[-1] / N))
hs.close()
src.free()
