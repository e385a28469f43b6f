"""HostStream under a tracer: N config-A batches submitted back to back (argv: N, mode slot|copyq),
for `rocprofv3 --kernel-trace --memory-copy-trace` timelines of the PCIe-inclusive pipeline."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "coeb-slam_amd"))
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
from coeb_front import HostBuffer, synth  # noqa: E402
from coeb_front.pipeline import HostStream  # noqa: E402

F, W, H = 257, 640, 480
N = int(sys.argv[1]) if len(sys.argv) > 1 else 12
mode = sys.argv[2] if len(sys.argv) > 2 else "slot"
fr = synth.make_frames(W, H, F, seed=1)
hs = HostStream(W, H, F, Tcw=np.stack([synth.motion_pose()] * F), mode=mode)
src = HostBuffer(F * H * W)
src.view(np.uint8, (F, H, W))[:] = fr
t0 = time.perf_counter()
sub = []
for i in range(N):
    ts = time.perf_counter()
    hs.submit(i, src)
    sub.append((time.perf_counter() - ts) * 1e3)
t1 = time.perf_counter()
hs.wait(N - 2)
hs.wait(N - 1)
print("submit ms: %s; all submitted after %.3f ms" % ([round(x, 3) for x in sub], (t1 - t0) * 1e3))
print("HostStream mode=%s: %d batches %.3f ms per batch" % (mode, N, (time.perf_counter() - t0) / N * 1e3))
hs.close()
