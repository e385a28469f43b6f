"""Diagnostic: raw H2D / D2H rates from page-locked memory, compute-only step, and the two-slot
HostStream step, on one 257-frame config-A batch."""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "coeb-slam_amd"))
import coeb_front as cf  # noqa: E402
from coeb_front import synth  # noqa: E402
from coeb_front.pipeline import BatchPipeline, HostStream  # noqa: E402

F, W, H = 257, 640, 480
fr = synth.make_frames(W, H, F, seed=1)
Tcw = np.stack([synth.motion_pose()] * F)
bp = BatchPipeline(W, H, F)
bp.load(fr, Tcw=Tcw)
src = cf.HostBuffer(F * H * W)
src.view(np.uint8, (F, H, W))[:] = fr
dst = cf.HostBuffer(F * H * W)
L, c = cf.lib(), bp.ctx


def timeit(fn, n=10):
    fn()
    c.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    c.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


nb = F * H * W
h2d = timeit(lambda: L.coeb_memcpy_h2d_async(c.h, C.c_void_p(bp.gray.ptr), C.c_void_p(src.ptr), nb))
d2h = timeit(lambda: L.coeb_memcpy_d2h_async(c.h, C.c_void_p(dst.ptr), C.c_void_p(bp.gray.ptr), nb))
comp = timeit(lambda: bp.run())
print("H2D %.3f ms (%.1f GB/s)  D2H %.3f ms (%.1f GB/s)  compute %.3f ms" % (h2d, nb / h2d / 1e6, d2h, nb / d2h / 1e6, comp))
both = timeit(lambda: (L.coeb_memcpy_h2d_async(c.h, C.c_void_p(bp.gray.ptr), C.c_void_p(src.ptr), nb), bp.run()))
print("H2D + compute same stream %.3f ms" % both)
bp2 = BatchPipeline(W, H, F)
bp2.load(fr, Tcw=Tcw)


def two():
    L.coeb_memcpy_h2d_async(c.h, C.c_void_p(bp.gray.ptr), C.c_void_p(src.ptr), nb)
    bp2.run()
    bp2.synchronize()


print("H2D on ctx A while ctx B computes: %.3f ms" % timeit(two))
if os.environ.get("DIAG_CLOSE"):
    bp2.close()
    bp.close()
hs = HostStream(W, H, F, Tcw=Tcw, shared_queue=bool(os.environ.get("HS_SHARED")))
for i in range(2):
    hs.submit(i, src)
hs.wait(0)
hs.wait(1)
for n in (10, 20, 40):
    t0 = time.perf_counter()
    for i in range(n):
        hs.submit(i, src)
    hs.wait(n - 2)
    hs.wait(n - 1)
    print("HostStream %d batches: %.3f ms per batch" % (n, (time.perf_counter() - t0) / n * 1e3))
# host-side time of each call inside submit (does something block the submitting thread?)
import coeb_front.pipeline as P  # noqa: E402
L = cf.lib()
orig = {}
for name in ("coeb_copyq_after_ctx", "coeb_copyq_h2d", "coeb_ctx_after_copyq", "coeb_copyq_d2h",
             "coeb_extract_batch_device", "coeb_match_batch_device_tcw", "coeb_copyq_synchronize"):
    orig[name] = getattr(L, name)
acc = {k: 0.0 for k in orig}


class Wrap:
    def __init__(self, k):
        self.k = k

    def __call__(self, *a):
        t = time.perf_counter()
        r = orig[self.k](*a)
        acc[self.k] += time.perf_counter() - t
        return r


class LP:
    def __getattr__(self, n):
        return Wrap(n) if n in orig else getattr(L, n)


P.lib = lambda: LP()
cf.lib = lambda: LP()
n = 20
t0 = time.perf_counter()
for i in range(n):
    hs.submit(i, src)
hs.wait(n - 2)
hs.wait(n - 1)
tt = (time.perf_counter() - t0) / n * 1e3
print("per batch %.3f ms; host ms per batch in: %s" % (tt, {k: round(v / n * 1e3, 3) for k, v in acc.items()}))
