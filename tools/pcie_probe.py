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
for q in qs:
    L.coeb_copyq_destroy(q)
ctx.close()
