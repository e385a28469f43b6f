"""CPU checks of the ProcessMovingObject oracle (Frame.cc:311-393): its canonical transcendental
functions against the host libm, solveCubic roots, pyrDown against an independent numpy
restatement, LK recovering a known shift, and the epipolar filter isolating a moving object.
OpenCV is not in the image, so these pin the restatement's behaviour, not OpenCV's bits
(parity vs OpenCV unpinned)."""
import math

import numpy as np
import pytest

from coeb_front import synth


@pytest.mark.parametrize("name,fn,lo,hi,tol", [("acos", math.acos, -1.0, 1.0, 1), ("exp", math.exp, -40, 40, 1),
                                               ("cos", math.cos, -8, 8, 2)])
def test_canonical_math(oracle_mod, name, fn, lo, hi, tol):
    xs = np.random.default_rng(1).uniform(lo, hi, 4000)
    for x in xs:
        a, b = oracle_mod.fd_math(name, float(x)), fn(float(x))
        assert abs(a - b) <= tol * math.ulp(b), (name, x, a, b)


def test_canonical_log(oracle_mod):
    for x in np.exp(np.random.default_rng(2).uniform(-600, 600, 4000)):
        a, b = oracle_mod.fd_math("log", float(x)), math.log(float(x))
        assert abs(a - b) <= math.ulp(b), (x, a, b)
    assert oracle_mod.fd_math("log", 1.0) == 0.0
    assert oracle_mod.fd_math("acos", 1.0) == 0.0


def test_solve_cubic(oracle_mod):
    n, r = oracle_mod.solve_cubic([1, -6, 11, -6])            # (x-1)(x-2)(x-3)
    assert n == 3 and np.allclose(sorted(r), [1, 2, 3], atol=1e-12)
    n, r = oracle_mod.solve_cubic([1, 0, 1, 1])                # one real root
    assert n == 1 and abs(r[0] ** 3 + r[0] + 1) < 1e-12
    n, r = oracle_mod.solve_cubic([0, 1, -3, 2])               # quadratic (x-1)(x-2)
    assert n == 2 and np.allclose(sorted(r[:2]), [1, 2])


def test_pyr_down_numpy(oracle_mod):
    img = np.random.default_rng(3).integers(0, 256, (61, 83), dtype=np.uint8)
    k = np.array([1, 4, 6, 4, 1])
    h, w = img.shape
    refl = lambda p, n: np.where(p < 0, -p, np.where(p >= n, 2 * n - 2 - p, p))
    ys = refl(np.arange((h + 1) // 2)[:, None] * 2 + np.arange(-2, 3)[None, :], h)
    xs = refl(np.arange((w + 1) // 2)[:, None] * 2 + np.arange(-2, 3)[None, :], w)
    acc = np.einsum("i,j,yixj->yx", k, k, img.astype(np.int64)[ys[:, :, None, None], xs[None, None, :, :]])
    assert np.array_equal(oracle_mod.pyr_down(img), ((acc + 128) >> 8).astype(np.uint8))


def test_lk_recovers_shift(oracle_mod):
    fr = synth.make_frames(640, 480, 2, seed=1001)
    pts = oracle_mod.corner_subpix(fr[0], oracle_mod.good_features(fr[0]))
    nx, st = oracle_mod.lk_pyr(fr[0], fr[1], pts)
    assert st.mean() > 0.9
    flow = np.median(nx[st == 1] - pts[st == 1], axis=0)
    assert np.allclose(flow, synth.SHIFT, atol=0.05), flow


def test_subpix_fast_and_edge_windows_agree(oracle_mod):
    """getRectSubPix's in-image path (the 8u32f recurrence) and its replicated-edge path are
    two formulas for one bilinear sample: they agree to float rounding."""
    import ctypes as C
    img = np.random.default_rng(4).integers(0, 256, (64, 64), dtype=np.uint8)
    lib = oracle_mod.lib()
    a = np.zeros(25 * 25, np.float32)
    lib.oc_rect_subpix_8u32f(oracle_mod.ptr(img), 64, 64, 64, 25, 25, C.c_float(30.3), C.c_float(31.7),
                             oracle_mod.ptr(a))
    ys, xs = np.mgrid[0:25, 0:25]
    fx, fy = 30.3 - 12 + xs, 31.7 - 12 + ys
    x0, y0 = np.floor(fx).astype(int), np.floor(fy).astype(int)
    ax, ay = fx - x0, fy - y0
    I = img.astype(np.float64)
    ref = ((1 - ax) * (1 - ay) * I[y0, x0] + ax * (1 - ay) * I[y0, x0 + 1] + (1 - ax) * ay * I[y0 + 1, x0] +
           ax * ay * I[y0 + 1, x0 + 1])
    assert np.abs(a.reshape(25, 25) - ref).max() < 1e-3


def test_fundamental_epipolar(oracle_mod):
    prev, cur, box = synth.moving_object_pair(640, 480, 1)
    pts = oracle_mod.corner_subpix(prev, oracle_mod.good_features(prev))
    nx, st = oracle_mod.lk_pyr(prev, cur, pts)
    tm, st2, F, nf = oracle_mod.moving_tail(prev, cur, pts, nx, st)
    assert F is not None and F[2, 2] == 1.0
    assert abs(np.linalg.det(F)) < 1e-6 * np.abs(F).max() ** 3 + 1e-12     # rank 2
    x0, y0, x1, y1 = box
    inb = (tm[:, 0] >= x0 - 2) & (tm[:, 0] < x1 + 2) & (tm[:, 1] >= y0 - 2) & (tm[:, 1] < y1 + 2)
    assert len(tm) >= 20 and inb.mean() > 0.8
    # fewer than 7 pairs: findFundamentalMat returns an empty Mat
    assert oracle_mod.find_fundamental(pts[:6], nx[:6]) is None


def test_static_scene_has_no_dynamic_points(oracle_mod):
    prev, cur, _ = synth.moving_object_pair(640, 480, 2, obj_shift=(2, 1))
    tm = oracle_mod.process_moving_object(prev, cur)
    assert tm is not None and len(tm) <= 5
