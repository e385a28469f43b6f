"""PCIe probe: page-locked host <-> device copy rates on one MI355X through the library's copy
queues (coeb_copyq_*), for the HostStream design: one 257-frame config-A upload
(79 MB) on 1 / 2 / 4 queues, the 17 MB result download alone, and both directions at once."""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "coeb-slam_amd"))
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
import coeb_front as cf  # noqa: E402

L = cf.lib()
ctx = cf.Context(1000, 1.2, 8, 20, 7)
UP = 257 * 640 * 480
DOWN = 17 * 1000 * 1000
hup, hdn = cf.HostBuffer(UP), cf.HostBuffer(DOWN)
dup, ddn = cf.DeviceBuffer(ctx, UP), cf.DeviceBuffer(ctx, DOWN)
qs = [L.coeb_copyq_create(ctx.h) for _ in range(4)]
assert all(qs), L.coeb_last_error(None)


def run(plan, reps=10):
    """plan: list of (queue index, 'h2d'|'d2h', offset, bytes); returns ms per repetition."""
    def once():
        for qi, kind, off, n in plan:
            if kind == "h2d":
                rc = L.coeb_copyq_h2d(qs[qi], C.c_void_p(dup.ptr + off), C.c_void_p(hup.ptr + off), n)
            else:
                rc = L.coeb_copyq_d2h(qs[qi], C.c_void_p(hdn.ptr + off), C.c_void_p(ddn.ptr + off), n)
            assert rc == 0, L.coeb_last_error(None)
        for q in set(p[0] for p in plan):
            assert L.coeb_copyq_synchronize(qs[q]) == 0
    once()
    t0 = time.perf_counter()
    for _ in range(reps):
        once()
    return (time.perf_counter() - t0) / reps * 1e3


def split(kind, total, k, q0=0):
    step = (total // k + 4095) & ~4095
    return [(q0 + i, kind, i * step, min(step, total - i * step)) for i in range(k) if i * step < total]


res = {}
for k in (1, 2, 4):
    ms = run(split("h2d", UP, k))
    res["h2d_%dq" % k] = ms
    print("H2D 79 MB on %d queue(s): %.3f ms  %.1f GB/s" % (k, ms, UP / ms / 1e6), flush=True)
ms = run(split("d2h", DOWN, 1))
print("D2H 17 MB on 1 queue: %.3f ms  %.1f GB/s" % (ms, DOWN / ms / 1e6), flush=True)
ms = run(split("d2h", DOWN, 2))
print("D2H 17 MB on 2 queues: %.3f ms  %.1f GB/s" % (ms, DOWN / ms / 1e6), flush=True)
ms = run(split("h2d", UP, 1) + [(1, "d2h", 0, DOWN)])
print("H2D 79 MB (q0) + D2H 17 MB (q1) at once: %.3f ms" % ms, flush=True)
ms = run(split("h2d", UP, 2) + [(2, "d2h", 0, DOWN)])
print("H2D 79 MB (q0,q1) + D2H 17 MB (q2) at once: %.3f ms" % ms, flush=True)
ms = run(split("h2d", UP, 1) + [(0, "d2h", 0, DOWN)])
print("H2D 79 MB then D2H 17 MB on one queue: %.3f ms" % ms, flush=True)

# copies beside the extraction kernels: compute alone, then an upload / download on the copy
# queues while a batch runs on another context, then HostStream with one shared or two queues
import numpy as np  # noqa: E402
from coeb_front import synth  # noqa: E402
from coeb_front.pipeline import BatchPipeline, HostStream  # noqa: E402
F, W, H = 257, 640, 480
fr = synth.make_frames(W, H, F, seed=1)
Tcw = np.stack([synth.motion_pose()] * F)
bp = BatchPipeline(W, H, F)
bp.load(fr, Tcw=Tcw)


def timed(fn, reps=10):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps * 1e3


def comp():
    bp.run()
    bp.synchronize()


print("compute alone: %.3f ms" % timed(comp), flush=True)


def comp_h2d():
    L.coeb_copyq_h2d(qs[0], C.c_void_p(dup.ptr), C.c_void_p(hup.ptr), UP)
    bp.run()
    bp.synchronize()
    L.coeb_copyq_synchronize(qs[0])


print("compute + H2D 79 MB beside it: %.3f ms" % timed(comp_h2d), flush=True)


def comp_both():
    L.coeb_copyq_h2d(qs[0], C.c_void_p(dup.ptr), C.c_void_p(hup.ptr), UP)
    L.coeb_copyq_d2h(qs[1], C.c_void_p(hdn.ptr), C.c_void_p(ddn.ptr), DOWN)
    bp.run()
    bp.synchronize()
    L.coeb_copyq_synchronize(qs[0])
    L.coeb_copyq_synchronize(qs[1])


print("compute + H2D 79 MB + D2H 17 MB beside it: %.3f ms" % timed(comp_both), flush=True)
bp2 = BatchPipeline(W, H, F)
bp2.load(fr, Tcw=Tcw)
c2 = bp2.ctx


def ctx_h2d_alone():
    L.coeb_memcpy_h2d_async(c2.h, C.c_void_p(bp2.gray.ptr), C.c_void_p(hup.ptr), UP)
    bp2.synchronize()


def ctx_h2d_beside():
    bp.run()
    L.coeb_memcpy_h2d_async(c2.h, C.c_void_p(bp2.gray.ptr), C.c_void_p(hup.ptr), UP)
    bp.synchronize()
    bp2.synchronize()


def ctx_h2d_then_run_beside():
    bp.run()
    L.coeb_memcpy_h2d_async(c2.h, C.c_void_p(bp2.gray.ptr), C.c_void_p(hup.ptr), UP)
    bp2.run()
    bp.synchronize()
    bp2.synchronize()


print("H2D on context B's stream alone: %.3f ms" % timed(ctx_h2d_alone), flush=True)
print("context A computes, H2D on context B's stream beside: %.3f ms" % timed(ctx_h2d_beside), flush=True)
print("context A computes, context B uploads then computes: %.3f ms" % timed(ctx_h2d_then_run_beside), flush=True)
bp2.close()
for q in qs:
    L.coeb_copyq_destroy(q)
src = cf.HostBuffer(F * H * W)
src.view(np.uint8, (F, H, W))[:] = fr
for mode, shared in (("ring", True), ("slot", True), ("copyq", True), ("copyq", False)):
    hs = HostStream(W, H, F, Tcw=Tcw, shared_queue=shared, mode=mode)
    for i in range(4):
        hs.submit(i, src)
    hs.wait(2)
    hs.wait(3)
    n = 30
    t0 = time.perf_counter()
    for i in range(n):
        hs.submit(i, src)
    hs.wait(n - 2)
    hs.wait(n - 1)
    ms = (time.perf_counter() - t0) / n * 1e3
    print("HostStream mode=%s shared_queue=%s: %.3f ms per batch, %.1f k frames/s" % (mode, shared, ms, 256 / ms),
          flush=True)
    hs.close()
ctx.close()
