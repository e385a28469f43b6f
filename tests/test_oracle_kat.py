"""Known-answer tests of the CPU oracle against the reference's own tables and definitions.

The reference ships no tests or golden vectors.  What it does hold are
constant tables and closed-form derived values; these pin the oracle:
  * bit_pattern_31_ (src/ORBextractor.cc:158-416), sha256 of the 1024 ints
  * umax (:461-476), features per level (:443-453), scale factors (:426-438)
  * pyramid level sizes (:1348-1349), SURVEY.md s8 level table
  * DescriptorDistance (src/ORBmatcher.cc:1648-1664) == popcount(a ^ b)
plus property checks of the OpenCV primitives the oracle restates.
"""
import hashlib
import math
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PATTERN_SHA = "88df8ca875cc8db56799edd57bb914edad8acb2d48c202b7a464a575b55dbdb8"


def inc_ints():
    txt = open(os.path.join(ROOT, "data", "orb_bit_pattern_31.inc")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return [int(v) for v in re.findall(r"-?\d+", txt)]


def test_pattern_table_pinned():
    vals = inc_ints()
    assert len(vals) == 1024
    assert hashlib.sha256(",".join(map(str, vals)).encode()).hexdigest() == PATTERN_SHA
    assert min(vals) >= -13 and max(vals) <= 12


@pytest.mark.skipif(not os.path.exists("/root/reference/src/ORBextractor.cc"), reason="reference not mounted")
def test_pattern_table_matches_reference_source():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from gen_pattern import extract
    assert extract() == inc_ints()


def test_oracle_pattern_loaded(oracle_mod):
    ex = oracle_mod.Extractor()
    pat = np.array(ex.p.pattern)
    assert pat.reshape(-1).tolist() == inc_ints()


def test_ctor_tables(oracle_mod):
    ex = oracle_mod.Extractor(1000, 1.2, 8, 20, 7)
    p = ex.p
    assert list(p.umax) == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]
    assert list(p.nfeat[:8]) == [217, 181, 151, 126, 105, 87, 73, 60]
    # mvScaleFactor[i] = (float)(mvScaleFactor[i-1] * (double)1.2f)
    s = [np.float32(1.0)]
    for i in range(1, 8):
        s.append(np.float32(np.float64(s[-1]) * np.float64(np.float32(1.2))))
    assert np.array_equal(np.array(p.scale[:8], np.float32), np.array(s, np.float32))
    B = oracle_mod.Extractor(2000, 1.2, 8, 20, 7)
    assert list(B.p.nfeat[:8]) == [434, 362, 302, 251, 209, 175, 145, 122]


def test_level_sizes_survey_table(oracle_mod):
    ex = oracle_mod.Extractor()
    assert ex.level_sizes(640, 480) == [(640, 480), (533, 400), (444, 333), (370, 278), (309, 231),
                                        (257, 193), (214, 161), (179, 134)]
    assert ex.level_sizes(1280, 960) == [(1280, 960), (1067, 800), (889, 667), (741, 556), (617, 463),
                                         (514, 386), (429, 322), (357, 268)]


def test_descriptor_distance_kat(oracle_mod):
    rng = np.random.default_rng(0)
    for _ in range(200):
        a = rng.integers(0, 256, 32, dtype=np.uint8)
        b = rng.integers(0, 256, 32, dtype=np.uint8)
        want = int(np.unpackbits(a ^ b).sum())
        assert oracle_mod.descriptor_distance(a, b) == want
    z = np.zeros(32, np.uint8)
    assert oracle_mod.descriptor_distance(z, np.full(32, 255, np.uint8)) == 256
    assert oracle_mod.descriptor_distance(z, z) == 0


def test_gauss_kernel_q8(oracle_mod):
    k = oracle_mod.gauss_kernel7()
    assert k == [18, 34, 48, 56, 48, 34, 18] and sum(k) == 256
    # exact float Gaussian, sigma 2, for reference: 0.07016, 0.13107, 0.19071, 0.21611
    g = np.exp(-np.arange(-3, 4) ** 2 / 8.0)
    g /= g.sum()
    assert np.abs(np.array(k) / 256.0 - g).max() < 2.5 / 256


def test_fast_atan2_properties(oracle_mod):
    f = oracle_mod.fast_atan2
    assert f(0.0, 0.0) == 0.0
    for deg in np.linspace(0, 359, 361):
        y, x = math.sin(math.radians(deg)), math.cos(math.radians(deg))
        a = f(y * 1000, x * 1000)
        d = (a - deg + 180) % 360 - 180
        assert abs(d) < 0.02, (deg, a)
        assert 0.0 <= a < 360.0 + 1e-4


def test_sincos_canonical_vs_libm(oracle_mod):
    """The canonical sincosf is the double-evaluated value rounded once to float: it must be
    within 1 ulp of the host libm sinf/cosf everywhere on [0, 2pi) and equal on >99.9%."""
    rng = np.random.default_rng(1)
    a = np.concatenate([rng.uniform(0, 2 * np.pi, 20000), np.linspace(0, 2 * np.pi, 5000)]).astype(np.float32)
    same = 0
    for v in a:
        s, c = oracle_mod.sincos(float(v))
        rs, rc = np.float32(math.sin(float(v))), np.float32(math.cos(float(v)))
        assert abs(int(np.float32(s).view(np.int32)) - int(rs.view(np.int32))) <= 1
        assert abs(int(np.float32(c).view(np.int32)) - int(rc.view(np.int32))) <= 1
        same += (np.float32(s) == rs) and (np.float32(c) == rc)
    assert same >= 0.999 * len(a)


def _corner_strength(patch):
    """Closed form used by the HIP k_fast: M = max over the 16 nine-pixel arcs of the
    arc's min of (v - ring) (dark) or (ring - v) (bright); corner at t <=> M > t and
    OpenCV cornerScore<16> = M - 1."""
    off = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3), (-2, -2),
           (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]
    v = int(patch[3, 3])
    d = [v - int(patch[3 + dy, 3 + dx]) for dx, dy in off]
    A = max(min(d[(k + j) % 16] for j in range(9)) for k in range(16))
    B = max(min(-d[(k + j) % 16] for j in range(9)) for k in range(16))
    return max(A, B)


def test_fast_closed_form_matches_opencv_literal(oracle_mod):
    """cv::FAST (literal restatement in the oracle) on a single-pixel ROI agrees with the
    closed form the GPU kernel evaluates, for many random and structured patches."""
    import ctypes as C
    L = oracle_mod.lib()
    rng = np.random.default_rng(2)
    xs = np.zeros(4, np.int32)
    ys = np.zeros(4, np.int32)
    sc = np.zeros(4, np.int32)
    checked = 0
    for it in range(6000):
        if it % 3 == 0:
            patch = rng.integers(0, 256, (7, 7)).astype(np.uint8)
        else:
            base = rng.integers(0, 256)
            patch = np.clip(base + rng.integers(-40, 41, (7, 7)), 0, 255).astype(np.uint8)
            if it % 3 == 2:
                patch[3, 3] = np.clip(int(patch[3, 3]) + rng.choice([-60, 60]), 0, 255)
        # embed in a 9x9 ROI so the centre pixel is the only detection candidate and NMS
        # neighbours are outside the detection window (score 0)
        roi = np.zeros((9, 9), np.uint8)
        roi[1:8, 1:8] = patch
        roi = np.ascontiguousarray(roi[1:8, 1:8])
        M = _corner_strength(roi)
        for t in (7, 10, 20, 30):
            n = L.oc_fast_roi(roi.ctypes.data_as(C.c_void_p), 7, 7, 7, t, xs.ctypes.data_as(C.c_void_p),
                              ys.ctypes.data_as(C.c_void_p), sc.ctypes.data_as(C.c_void_p), 4)
            if M > t:
                assert n == 1 and sc[0] == M - 1, (t, M, n, sc[0])
                checked += 1
            else:
                assert n == 0
    assert checked > 500


def test_resize_and_blur_constant_images(oracle_mod):
    """resize / blur of a constant image stay constant (fixed-point weights sum to 1)."""
    ex = oracle_mod.Extractor()
    for v in (0, 1, 77, 128, 254, 255):
        img = np.full((480, 640), v, np.uint8)
        r = ex.extract(img, debug=True)
        assert (r["pyramid"] == v).all()
        assert len(r["kps"]) == 0


# ---- local-map SearchByProjection: C oracle vs a literal Python loop (ORBmatcher.cc:44-129) ----
def _py_search_local_map(cam, kps, desc, ur, cur_obs, mp, th, nnratio):
    """Pure-Python restatement, small sizes only: AssignFeaturesToGrid (Frame.cc:396-411,
    PosInGrid :553-568), GetFeaturesInArea (:503-551), the search loop (ORBmatcher.cc:44-129)."""
    f32 = np.float32
    cols, rows = 64, 48
    grid = [[[] for _ in range(rows)] for _ in range(cols)]
    for i, k in enumerate(kps):
        px = math.floor(abs(float((f32(k["x"]) - cam.min_x) * f32(cam.grid_inv_w))) + 0.5)
        py = math.floor(abs(float((f32(k["y"]) - cam.min_y) * f32(cam.grid_inv_h))) + 0.5)
        if (f32(k["x"]) - cam.min_x) < 0:
            px = -px
        if (f32(k["y"]) - cam.min_y) < 0:
            py = -py
        if 0 <= px < cols and 0 <= py < rows:
            grid[px][py].append(i)

    def in_area(x, y, r, minL, maxL):
        out = []
        x0 = max(0, math.floor(float((f32(x) - f32(cam.min_x) - f32(r)) * f32(cam.grid_inv_w))))
        if x0 >= cols:
            return out
        x1 = min(cols - 1, math.ceil(float((f32(x) - f32(cam.min_x) + f32(r)) * f32(cam.grid_inv_w))))
        if x1 < 0:
            return out
        y0 = max(0, math.floor(float((f32(y) - f32(cam.min_y) - f32(r)) * f32(cam.grid_inv_h))))
        if y0 >= rows:
            return out
        y1 = min(rows - 1, math.ceil(float((f32(y) - f32(cam.min_y) + f32(r)) * f32(cam.grid_inv_h))))
        if y1 < 0:
            return out
        chk = minL > 0 or maxL >= 0
        for ix in range(x0, x1 + 1):
            for iy in range(y0, y1 + 1):
                for j in grid[ix][iy]:
                    if chk and (kps[j]["octave"] < minL or (maxL >= 0 and kps[j]["octave"] > maxL)):
                        continue
                    if abs(f32(kps[j]["x"]) - f32(x)) < f32(r) and abs(f32(kps[j]["y"]) - f32(y)) < f32(r):
                        out.append(j)
        return out

    holder = list(cur_obs)
    match = [-1] * len(kps)
    nm = 0
    for q in range(len(mp["in_view"])):
        if not mp["in_view"][q]:
            continue
        lvl = int(mp["level"][q])
        r = f32(2.5) if f32(mp["view_cos"][q]) > f32(0.998) else f32(4.0)
        if th != 1.0:
            r = f32(r * f32(th))
        rs = f32(r * f32(cam.scale[lvl]))
        best, bl, best2, bl2, bi = 256, -1, 256, -1, -1
        for idx in in_area(mp["proj_x"][q], mp["proj_y"][q], rs, lvl - 1, lvl):
            if holder[idx] > 0:
                continue
            if ur[idx] > 0 and abs(f32(mp["proj_xr"][q]) - f32(ur[idx])) > rs:
                continue
            d = sum(bin(int(a) ^ int(b)).count("1") for a, b in zip(mp["descriptor"][q], desc[idx]))
            if d < best:
                best2, bl2, best, bl, bi = best, bl, d, int(kps[idx]["octave"]), idx
            elif d < best2:
                bl2, best2 = int(kps[idx]["octave"]), d
        if best <= 100:
            if bl == bl2 and f32(best) > f32(nnratio) * f32(best2):
                continue
            match[bi] = q
            holder[bi] = int(mp["observations"][q])
            nm += 1
    return nm, np.array(match, np.int32)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_search_local_map_oracle_vs_python(oracle_mod, seed):
    rng = np.random.default_rng(seed)
    ex = oracle_mod.Extractor()
    cam = oracle_mod.camera(ex, 640, 480, 535.4, 539.2, 320.1, 247.6, 40.0)
    n, m = 300, 260
    kps = np.zeros(n, oracle_mod.KP_DTYPE)
    kps["x"] = rng.uniform(0, 640, n)
    kps["y"] = rng.uniform(0, 480, n)
    kps["octave"] = rng.integers(0, 8, n)
    desc = rng.integers(0, 256, (n, 32)).astype(np.uint8)
    ur = np.where(rng.random(n) < 0.7, kps["x"] - rng.uniform(5, 30, n), -1).astype(np.float32)
    cur_obs = rng.choice(np.array([-1, -1, 0, 2], np.int32), n).astype(np.int32)
    src = rng.integers(0, n, m)
    d = desc[src].copy()
    flip = rng.integers(0, 256, (m, 30))
    for q in range(m):                       # 0..30 flipped bits: near and far descriptors
        for b in flip[q, : rng.integers(0, 31)]:
            d[q, b >> 3] ^= np.uint8(1 << (b & 7))
    px = (kps["x"][src] + rng.normal(0, 3, m)).astype(np.float32)
    mp = dict(in_view=(rng.random(m) < 0.9).astype(np.uint8), proj_x=px,
              proj_y=(kps["y"][src] + rng.normal(0, 3, m)).astype(np.float32),
              proj_xr=(px - rng.uniform(5, 30, m)).astype(np.float32),
              level=np.clip(kps["octave"][src] + rng.integers(-1, 2, m), 0, 7).astype(np.int32),
              view_cos=rng.uniform(0.99, 1.0, m).astype(np.float32), descriptor=d,
              observations=rng.choice(np.array([0, 1, 2], np.int32), m).astype(np.int32))
    for th, ratio in ((3.0, 0.8), (1.0, 1.0), (6.0, 0.6)):
        nm, mt = oracle_mod.search_local_map(cam, kps, desc, ur, cur_obs, mp, th, ratio)
        nm_py, mt_py = _py_search_local_map(cam, kps, desc, ur, cur_obs, mp, th, ratio)
        assert nm == nm_py and np.array_equal(mt, mt_py)
        assert nm > 0


# ---- relocalisation SearchByProjection: C oracle vs a literal Python loop (ORBmatcher.cc:1473-1600) ----
def _py_search_keyframe(cam, kps, desc, cur_has, kf, T, th, orb_dist, check_ori):
    f32, f64 = np.float32, np.float64
    cols, rows = 64, 48
    grid = [[[] for _ in range(rows)] for _ in range(cols)]
    for i, k in enumerate(kps):
        gx = float((f32(k["x"]) - f32(cam.min_x)) * f32(cam.grid_inv_w))
        gy = float((f32(k["y"]) - f32(cam.min_y)) * f32(cam.grid_inv_h))
        px = int(math.copysign(math.floor(abs(gx) + 0.5), gx))
        py = int(math.copysign(math.floor(abs(gy) + 0.5), gy))
        if 0 <= px < cols and 0 <= py < rows:
            grid[px][py].append(i)
    T = np.asarray(T, f32)
    Ow = [f32(-(f64(T[0, k]) * f64(T[0, 3]) + f64(T[1, k]) * f64(T[1, 3]) + f64(T[2, k]) * f64(T[2, 3])))
          for k in range(3)]
    log_sf = f32(math.log(f64(f32(cam.scale[1]))))
    taken = [bool(h) for h in cur_has]
    match = [-1] * len(kps)
    hist = []
    nm = 0
    for q in range(len(kf["valid"])):
        if not kf["valid"][q]:
            continue
        X = kf["world_pos"][q].astype(f32)
        p3 = []
        for k in range(3):
            t = f32(T[k, 0] * X[0]) + f32(T[k, 1] * X[1])
            t = f32(t + f32(T[k, 2] * X[2]))
            p3.append(f32(f64(t) + f64(T[k, 3])))
        invz = f32(1.0 / f64(p3[2]))
        u = f32(f64(f32(f32(cam.fx) * p3[0])) * f64(invz) + f64(f32(cam.cx)))    # fmaf, exact in double
        v = f32(f64(f32(f32(cam.fy) * p3[1])) * f64(invz) + f64(f32(cam.cy)))
        if u < f32(cam.min_x) or u > f32(cam.max_x) or v < f32(cam.min_y) or v > f32(cam.max_y):
            continue
        d = [f32(X[k] - Ow[k]) for k in range(3)]
        ss = 0.0
        for k in range(3):
            ss += f64(d[k]) * f64(d[k])
        dist3 = f32(math.sqrt(ss))
        if dist3 < f32(f32(0.8) * f32(kf["min_distance"][q])) or dist3 > f32(f32(1.2) * f32(kf["max_distance"][q])):
            continue
        ratio = f32(f32(kf["max_distance"][q]) / dist3)
        lvl = int(math.ceil(f32(f32(math.log(f64(ratio))) / log_sf)))
        lvl = min(max(lvl, 0), cam.nlevels - 1)
        r = f32(f32(th) * f32(cam.scale[lvl]))
        x0 = max(0, math.floor(f32(f32(u - f32(cam.min_x)) - r) * f32(cam.grid_inv_w)))
        x1 = min(cols - 1, math.ceil(f32(f32(u - f32(cam.min_x)) + r) * f32(cam.grid_inv_w)))
        y0 = max(0, math.floor(f32(f32(v - f32(cam.min_y)) - r) * f32(cam.grid_inv_h)))
        y1 = min(rows - 1, math.ceil(f32(f32(v - f32(cam.min_y)) + r) * f32(cam.grid_inv_h)))
        if x0 >= cols or x1 < 0 or y0 >= rows or y1 < 0:
            continue
        best, bi = 256, -1
        for ix in range(x0, x1 + 1):
            for iy in range(y0, y1 + 1):
                for j in grid[ix][iy]:
                    o = int(kps[j]["octave"])
                    if o < lvl - 1 or o > lvl + 1:
                        continue
                    if not (abs(f32(kps[j]["x"]) - u) < r and abs(f32(kps[j]["y"]) - v) < r):
                        continue
                    if taken[j]:
                        continue
                    dd = sum(bin(int(a) ^ int(b)).count("1") for a, b in zip(kf["descriptor"][q], desc[j]))
                    if dd < best:
                        best, bi = dd, j
        if best <= orb_dist:
            taken[bi] = True
            match[bi] = q
            nm += 1
            if check_ori:
                rot = f32(f32(kf["angle"][q]) - f32(kps[bi]["angle"]))
                if rot < 0:
                    rot = f32(rot + f32(360.0))
                x = float(f32(rot * f32(1.0 / 30)))
                b = int(math.floor(x + 0.5))
                hist.append((bi, 0 if b == 30 else b))
    if check_ori:
        h = [0] * 30
        for _, b in hist:
            h[b] += 1
        m1 = m2 = m3 = 0
        i1 = i2 = i3 = -1
        for i in range(30):
            if h[i] > m1:
                m3, m2, m1, i3, i2, i1 = m2, m1, h[i], i2, i1, i
            elif h[i] > m2:
                m3, m2, i3, i2 = m2, h[i], i2, i
            elif h[i] > m3:
                m3, i3 = h[i], i
        if m2 < f32(0.1) * f32(m1):
            i2 = i3 = -1
        elif m3 < f32(0.1) * f32(m1):
            i3 = -1
        for bi, b in hist:
            if b not in (i1, i2, i3):
                match[bi] = -1
                nm -= 1
    return nm, np.array(match, np.int32)


@pytest.mark.parametrize("seed", [0, 1])
def test_search_keyframe_oracle_vs_python(oracle_mod, seed):
    rng = np.random.default_rng(seed)
    ex = oracle_mod.Extractor()
    cam = oracle_mod.camera(ex, 640, 480, 535.4, 539.2, 320.1, 247.6, 40.0)
    n, m = 300, 260
    kps = np.zeros(n, oracle_mod.KP_DTYPE)
    kps["x"] = rng.uniform(0, 640, n)
    kps["y"] = rng.uniform(0, 480, n)
    kps["octave"] = rng.integers(0, 8, n)
    kps["angle"] = rng.uniform(0, 360, n)
    desc = rng.integers(0, 256, (n, 32)).astype(np.uint8)
    src = rng.integers(0, n, m)
    z = rng.uniform(1.0, 4.0, m).astype(np.float32)
    xw = np.stack([((kps["x"][src] + rng.normal(0, 2, m) - 320.1) * z / 535.4),
                   ((kps["y"][src] + rng.normal(0, 2, m) - 247.6) * z / 539.2), z], 1).astype(np.float32)
    d = desc[src].copy()
    for q in range(m):
        for b in rng.integers(0, 256, rng.integers(0, 40)):
            d[q, b >> 3] ^= np.uint8(1 << (b & 7))
    dist = np.sqrt((xw.astype(np.float64) ** 2).sum(1)).astype(np.float32)
    maxd = (dist * np.float32(1.2) ** kps["octave"][src].astype(np.float32) * rng.uniform(0.9, 1.1, m)).astype(np.float32)
    kf = dict(valid=(rng.random(m) < 0.9).astype(np.uint8), world_pos=xw, descriptor=d, max_distance=maxd,
              min_distance=(maxd / np.float32(1.2) ** 7).astype(np.float32),
              angle=(kps["angle"][src] + rng.normal(0, 5, m)).astype(np.float32) % 360)
    T = np.eye(4, dtype=np.float32)
    T[:3, 3] = [0.01, -0.02, 0.015]
    has = (rng.random(n) < 0.2).astype(np.uint8)
    for th, od, ori in ((10.0, 100, True), (3.0, 64, True), (15.0, 80, False)):
        nm, mt = oracle_mod.search_keyframe(cam, kps, desc, has, kf, T, th, od, ori)
        nm_py, mt_py = _py_search_keyframe(cam, kps, desc, has, kf, T, th, od, ori)
        assert nm == nm_py and np.array_equal(mt, mt_py), (nm, nm_py)
        assert nm > 0


# ---- Optimizer::PoseOptimization oracle: properties (g2o absent: parity vs g2o unpinned) ----
def _inv_sigma2(nlevels=8, sf=1.2):
    s = [np.float32(1.0)]
    for _ in range(1, nlevels):
        s.append(np.float32(np.float64(s[-1]) * sf))
    return np.array([np.float32(1.0) / np.float32(x * x) for x in s], np.float32)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_pose_optimization_oracle_recovers_pose(oracle_mod, seed):
    from coeb_front import synth
    P = synth.make_pose_problem(seed=seed)
    nin, T, outl = oracle_mod.pose_optimization(P["kps"], P["has_mp"], P["xw"], P["ur"], _inv_sigma2(),
                                                535.4, 539.2, 320.1, 247.6, 40.0, P["Tcw_init"])
    Tt = P["Tcw_true"].astype(np.float64)
    dR = T[:3, :3].astype(np.float64) @ Tt[:3, :3].T
    ang = np.arccos(np.clip((np.trace(dR) - 1) / 2, -1, 1))
    assert ang < 2e-3 and np.linalg.norm(T[:3, 3] - Tt[:3, 3]) < 5e-3, (ang, T[:3, 3], Tt[:3, 3])
    has = P["has_mp"] > 0
    gross = P["gross"] & has
    assert outl[gross].mean() > 0.9                 # gross outliers classified
    assert outl[has & ~P["gross"]].mean() < 0.1     # inliers kept
    assert nin == int(has.sum() - outl[has].sum())


def test_pose_optimization_oracle_edge_cases(oracle_mod):
    from coeb_front import synth
    P = synth.make_pose_problem(n=40, seed=5)
    has = np.zeros_like(P["has_mp"])
    has[:2] = 1                                     # < 3 correspondences: pose untouched, 0
    nin, T, outl = oracle_mod.pose_optimization(P["kps"], has, P["xw"], P["ur"], _inv_sigma2(),
                                                535.4, 539.2, 320.1, 247.6, 40.0, P["Tcw_init"])
    assert nin == 0 and np.array_equal(T, P["Tcw_init"])
    has[:8] = 1                                     # < 10 edges: a single round
    nin, T, outl = oracle_mod.pose_optimization(P["kps"], has, P["xw"], P["ur"], _inv_sigma2(),
                                                535.4, 539.2, 320.1, 247.6, 40.0, P["Tcw_init"])
    assert 0 < nin <= 8


def exact_pose_problem(n_side=8):
    """A PoseOptimization input whose residuals are exactly zero at the entry pose (identity):
    dyadic 3-D points, fx = fy = 512, integer principal point, depth 1 or 2, so every projection,
    disparity and error is exact in float and double.  Then b = 0, the LM step is x = 0 and
    tempChi == currentChi: g2o's `scale += 1e-3` makes rho exactly 0 -> Terminate after one
    iteration per round (without it rho = 0/0 = NaN and all 10 iterations run)."""
    from coeb_front import KEYPOINT_DTYPE
    pts, kps = [], []
    for i in range(n_side):
        for j in range(n_side):
            z = 1.0 if (i + j) % 2 else 2.0
            X, Y = (i - n_side / 2) / 8.0, (j - n_side / 2) / 16.0
            pts.append((X, Y, z))
            kps.append((512.0 * X / z + 320.0, 512.0 * Y / z + 240.0))
    n = len(pts)
    k = np.zeros(n, KEYPOINT_DTYPE)
    k["x"], k["y"] = np.array(kps, np.float32).T
    k["octave"] = np.arange(n) % 8
    k["class_id"] = -1
    xw = np.array(pts, np.float32)
    ur = (k["x"] - np.float32(40.0) / xw[:, 2]).astype(np.float32)
    ur[::3] = -1.0                                   # a third monocular
    return dict(kps=k, has_mp=np.ones(n, np.uint8), xw=xw, ur=ur, Tcw_init=np.eye(4, dtype=np.float32),
                cam=(512.0, 512.0, 320.0, 240.0, 40.0))


def test_pose_optimization_rho_zero_terminates(oracle_mod):
    """g2o's OptimizationAlgorithmLevenberg::solve adds 1e-3 to computeScale() before
    dividing; at a zero-residual optimum rho == 0 must end each round after one iteration."""
    P = exact_pose_problem()
    nin, T, outl = oracle_mod.pose_optimization(P["kps"], P["has_mp"], P["xw"], P["ur"], _inv_sigma2(), *P["cam"],
                                                P["Tcw_init"])
    assert nin == len(P["kps"]) and not outl.any()
    assert np.array_equal(T, np.eye(4, dtype=np.float32))
    assert oracle_mod.pose_last_stats() == (4, 4)     # 4 rounds x (1 iteration, 1 trial)
    # a perturbed start converges (rho > 0 steps) and is not cut short
    T0 = np.eye(4, dtype=np.float32)
    T0[0, 3] = 0.01
    nin, T, _ = oracle_mod.pose_optimization(P["kps"], P["has_mp"], P["xw"], P["ur"], _inv_sigma2(), *P["cam"], T0)
    it, tr = oracle_mod.pose_last_stats()
    assert nin == len(P["kps"]) and abs(T[0, 3]) < 1e-5 and it > 4 and tr >= it


# ---- Frame::UndistortKeyPoints oracle: distort -> undistort round trip ----
TUM1_DIST = (0.262383, -0.953104, -0.005358, 0.002628, 1.163314)   # Examples/RGB-D/TUM1.yaml


def test_undistort_oracle_round_trip(oracle_mod):
    rng = np.random.default_rng(3)
    fx, fy, cx, cy = 517.306408, 516.469215, 318.643040, 255.313989
    k1, k2, p1, p2, k3 = TUM1_DIST
    n = 500
    xn = rng.uniform(-0.35, 0.35, n)
    yn = rng.uniform(-0.3, 0.3, n)
    r2 = xn * xn + yn * yn
    rad = 1 + k1 * r2 + k2 * r2 * r2 + k3 * r2 ** 3
    xd = xn * rad + 2 * p1 * xn * yn + p2 * (r2 + 2 * xn * xn)
    yd = yn * rad + p1 * (r2 + 2 * yn * yn) + 2 * p2 * xn * yn
    kps = np.zeros(n, oracle_mod.KP_DTYPE)
    kps["x"] = fx * xd + cx
    kps["y"] = fy * yd + cy
    kps["octave"] = rng.integers(0, 8, n)
    un = oracle_mod.undistort_keypoints(kps, fx, fy, cx, cy, TUM1_DIST)
    err = np.hypot(un["x"] - (fx * xn + cx), un["y"] - (fy * yn + cy))
    assert np.median(err) < 0.01 and err.max() < 0.5, (np.median(err), err.max())
    assert np.array_equal(un["octave"], kps["octave"])
    same = oracle_mod.undistort_keypoints(kps, fx, fy, cx, cy, (0.0, 0.1, 0.1, 0.1, 0.1))   # k1 == 0: copy
    assert np.array_equal(same, kps)


def test_tum_association_golden():
    """coeb_tum_read_list + coeb_tum_associate (host C++ behind the C-ABI) vs the reference
    associate.py's own output on the same lists (tests/golden/make_tum_golden.py)."""
    import json
    import coeb_front
    cases = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "tum_assoc.json")))
    for c in cases:
        rgb, depth = coeb_front.tum_read_file_list(c["rgb"]), coeb_front.tum_read_file_list(c["depth"])
        got = coeb_front.tum_associate(rgb, depth, c["offset"], c["max_difference"])
        assert [list(x) for x in got] == c["matches"]
        assert len(got) > 20
        assert all(len(v) >= 1 for v in rgb.values())


def test_tum_association_reference_files():
    """The reference's own association outputs (Examples/RGB-D/associations/*.txt: 11 TUM
    sequences, 18,520 pairs that associate.py:49-102 produced with offset 0, max_difference 0.02),
    re-derived through the C-ABI: each file is read with coeb_tum_read_list, split into its rgb
    and depth stamp lists, and re-associated with coeb_tum_associate.  Greedy selection restricted
    to the matched stamps takes exactly the original pairs (every candidate among them is a
    candidate of the full run at the same rank, and the pairs that blocked it there are matched
    pairs too), so every file must come back identical, in its own order.  Fixture packed by
    tests/golden/make_tum_assoc_files.py."""
    import coeb_front
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "tum_assoc_files.npz"))
    assert len(z.files) == 11
    total = 0
    for name in sorted(z.files):
        text = z[name].tobytes().decode()
        lines = [ln.split() for ln in text.splitlines() if ln.strip() and not ln.startswith("#")]
        want = [(float(r[0]), float(r[2])) for r in lines]
        # the association file itself through the C-ABI reader: stamp = rgb stamp, data = the rest
        assoc = coeb_front.tum_read_file_list(text)
        assert list(assoc.keys()) == [a for a, _ in want], name
        rgb_text = "".join("%s %s\n" % (a, v[0]) for a, v in zip((r[0] for r in lines), assoc.values()))
        depth_text = "".join("%s %s\n" % (v[1], v[2]) for v in assoc.values())
        rgb, depth = coeb_front.tum_read_file_list(rgb_text), coeb_front.tum_read_file_list(depth_text)
        assert len(rgb) == len(depth) == len(lines), name
        got = coeb_front.tum_associate(rgb, depth, 0.0, 0.02)
        assert got == want, name
        total += len(got)
    assert total == 18520, total


def test_tum_stamp_parse_ignores_process_locale():
    """coeb_tum_read_list parses stamps in the "C" locale, as Python's float() does, even after
    the host process switched LC_NUMERIC to a comma-decimal locale."""
    import ctypes as C
    import ctypes.util
    import coeb_front
    libc = C.CDLL(ctypes.util.find_library("c"))
    libc.setlocale.restype = C.c_char_p
    LC_NUMERIC = 1
    old = libc.setlocale(LC_NUMERIC, None)
    switched = None
    for loc in (b"de_DE.UTF-8", b"de_DE.utf8", b"fr_FR.UTF-8", b"ru_RU.UTF-8"):
        switched = libc.setlocale(LC_NUMERIC, loc)
        if switched:
            break
    try:
        lst = coeb_front.tum_read_file_list("1305031102.175304 rgb/a.png\n1305031102.211214 rgb/b.png\n")
        assert list(lst.keys()) == [1305031102.175304, 1305031102.211214]
    finally:
        libc.setlocale(LC_NUMERIC, old)
    if not switched:
        pytest.skip("no comma-decimal locale installed: parsed in the default locale only")


def test_tum_association_edge_cases():
    """The association's definition on hand cases: greedy by (difference, a, b), each stamp once,
    the strict < max_difference bound, offset applied to the second list, ties on the difference
    broken by a then b, duplicates / NaN / comments / short lines in the lists."""
    import coeb_front
    A = coeb_front.tum_associate
    assert A([], [1.0]) == [] and A([1.0], []) == []
    assert A([1.0, 2.0], [1.01, 1.99]) == [(1.0, 1.01), (2.0, 1.99)]
    assert A([1.0], [1.02]) == []                                   # |d| == 0.02 is not < 0.02
    assert A([1.0], [1.015]) == [(1.0, 1.015)]
    assert A([1.0, 1.02], [1.01]) == [(1.0, 1.01)]                  # equal |d|: smaller a first
    assert A([1.01], [1.0, 1.02]) == [(1.01, 1.0)]                  # equal |d| and a: smaller b first
    assert A([1.0, 1.011], [1.01]) == [(1.011, 1.01)]               # greedy: the closer pair wins
    assert A([5.0], [4.5], offset=0.5) == [(5.0, 4.5)]
    assert A([1.0, 1.0], [1.0]) == [(1.0, 1.0)]                     # a stamp given twice is one stamp
    assert A([float("nan"), 1.0], [float("nan"), 1.0]) == [(1.0, 1.0)]
    rng = np.random.default_rng(7)
    a = np.sort(rng.uniform(0, 30, 900)).round(6)
    b = np.sort(a + rng.normal(0, 0.01, a.size)).round(6)
    got = A(a, b, 0.003, 0.02)
    # brute force of the definition
    cand = sorted((abs(x - (y + 0.003)), x, y) for x in set(a.tolist()) for y in set(b.tolist())
                  if abs(x - (y + 0.003)) < 0.02)
    ua, ub, want = set(), set(), []
    for _, x, y in cand:
        if x not in ua and y not in ub:
            ua.add(x), ub.add(y), want.append((x, y))
    assert got == sorted(want) and len(got) > 500
    text = "# c\n1.5 rgb/a.png\n\n2.5,rgb/b.png x\n3.5\n #x\n".replace(" #x\n", "")
    lst = coeb_front.tum_read_file_list(text + "2.5\trgb/c.png\n")
    assert lst == {1.5: ["rgb/a.png"], 2.5: ["rgb/c.png"]}
    with pytest.raises(coeb_front.CoebError):
        coeb_front.tum_read_file_list("x.png 1.0\n")               # read_file_list's float() raises


def test_grab_image_rgbd_conversions_kat(oracle_mod):
    """GrabImageRGBD's cvtColor (Tracking.cc:212-225): the OpenCV 3.4 8U coefficients give the
    well-known gray levels of the primaries (R -> 76, G -> 150, B -> 29); RGB vs BGR swap R and
    B; the 4-channel forms ignore alpha; a gray image is used as is.  Depth (:227-228): 16UC1
    scaled in float; 32FC1 with factor 1 unchanged (NaN and -0 included)."""
    px = np.array([[[255, 0, 0], [0, 255, 0], [0, 0, 255], [255, 255, 255]]], np.uint8)
    assert oracle_mod.image_to_gray(px, 1).tolist() == [[76, 150, 29, 255]]
    assert oracle_mod.image_to_gray(px, 0).tolist() == [[29, 150, 76, 255]]
    rgba = np.concatenate([px, np.array([[[0], [17], [128], [255]]], np.uint8)], axis=2)
    assert oracle_mod.image_to_gray(rgba, 1).tolist() == [[76, 150, 29, 255]]
    g = np.arange(12, dtype=np.uint8).reshape(3, 4)
    assert np.array_equal(oracle_mod.image_to_gray(g), g)
    d16 = np.array([[0, 1, 5000, 65535]], np.uint16)
    f = np.float32(1 / 5000.0)
    assert np.array_equal(oracle_mod.depth_to_float(d16, f), d16.astype(np.float32) * f)
    d32 = np.array([[np.nan, -0.0, 1.5, 3e38]], np.float32)
    assert np.array_equal(oracle_mod.depth_to_float(d32, 1.0).view(np.uint32), d32.view(np.uint32))
    assert np.array_equal(oracle_mod.depth_to_float(d32, 2.0)[0, 2:], np.float32([3.0, np.inf]))


@pytest.mark.timeout(300)
def test_oracle_clean_under_asan_ubsan():
    """The oracle built with AddressSanitizer + UndefinedBehaviorSanitizer (no recovery) runs every
    public entry point on synthetic frames without a finding (`make -C oracle asan`, kat_main.c)."""
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run(["make", "-s", "-C", os.path.join(root, "oracle"), "asan"], capture_output=True, text=True,
                       timeout=280)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "kat_main: clean" in r.stdout


def _py_resize_linear(src, dw, dh):
    """numpy restatement of OpenCV 3.4 resize INTER_LINEAR 8U on x86-64 (imgproc resize.cpp):
    11-bit coefficient tables, exact horizontal pass, vertical pass with the SSE2 rounding of
    VResizeLinearVec_32s8u up to its last column and FixedPtCast<int,uchar,22> after it."""
    sh, sw = src.shape
    sx_scale, sy_scale = 1.0 / (dw / sw), 1.0 / (dh / sh)

    def tab(n, scale, limit):
        ofs, c0, c1, xmax = [], [], [], n
        for d in range(n):
            f = np.float32((d + 0.5) * scale - 0.5)
            s = int(np.floor(f))
            f = np.float32(f - np.float32(s))
            if limit:
                if s < 0:
                    f, s = np.float32(0), 0
                if s + 1 >= sw:
                    xmax = min(xmax, d)
                    if s >= sw - 1:
                        f, s = np.float32(0), sw - 1
            ofs.append(s)
            c0.append(int(np.rint(np.float32(np.float32(1) - f) * np.float32(2048))))     # cvRound, half even
            c1.append(int(np.rint(np.float32(f) * np.float32(2048))))
        return np.array(ofs), np.array(c0), np.array(c1), xmax
    xofs, a0, a1, xmax = tab(dw, sx_scale, True)
    yofs, b0, b1, _ = tab(dh, sy_scale, False)
    x = (dw // 16) * 16 if dw >= 16 else 0
    while x < dw - 4:
        x += 4
    out = np.zeros((dh, dw), np.uint8)
    s = src.astype(np.int64)
    for dy in range(dh):
        r0 = min(max(yofs[dy], 0), sh - 1)
        r1 = min(max(yofs[dy] + 1, 0), sh - 1)
        h = []
        for r in (r0, r1):
            row = s[r]
            hx = np.where(np.arange(dw) < xmax, row[xofs] * a0 + row[np.minimum(xofs + 1, sw - 1)] * a1, row[xofs] * 2048)
            h.append(hx)
        simd = (((h[0] >> 4) * b0[dy]) >> 16) + (((h[1] >> 4) * b1[dy]) >> 16)
        simd = (simd + 2) >> 2
        exact = (h[0] * b0[dy] + h[1] * b1[dy] + (1 << 21)) >> 22
        v = np.where(np.arange(dw) < x, simd, exact)
        out[dy] = np.clip(v, 0, 255)
    return out


def test_resize_linear_simd_prefix_scalar_tail(oracle_mod):
    """The oracle's resize matches the numpy restatement on every ORB level size of configs A and
    B, including the columns after the SSE2 loops (1 to 4 per row: 533 -> 1, 444 -> 4, ...)."""
    import ctypes as C
    rng = np.random.default_rng(5)
    src = rng.integers(0, 256, (480, 640), dtype=np.uint8)
    for dw, dh in ((533, 400), (444, 333), (370, 278), (309, 231), (179, 134), (641 // 2, 479 // 2)):
        ref = _py_resize_linear(src, dw, dh)
        out = np.zeros((dh, dw), np.uint8)
        oracle_mod.lib().oc_resize_linear(src.ctypes.data_as(C.c_void_p), 640, 480, 640, out.ctypes.data_as(C.c_void_p),
                                          dw, dh, dw)
        assert np.array_equal(out, ref), (dw, dh)
        tail = oracle_mod.lib().oc_resize_simd_end(dw)
        assert dw - 4 <= tail <= dw
    # the scalar tail rounds differently from the SIMD form on some inputs
    assert any(oracle_mod.lib().oc_resize_simd_end(w) < w for w in (533, 444, 370, 309))


def _frustum(O, cam, T, P, Pn, maxd, mind):
    import ctypes as C
    px, py, pxr, vc = C.c_float(), C.c_float(), C.c_float(), C.c_float()
    lvl = C.c_int32()
    f3 = lambda v: np.ascontiguousarray(v, np.float32)   # noqa: E731
    P, Pn, T = f3(P), f3(Pn), f3(T)
    ok = O.lib().oc_is_in_frustum(C.byref(cam), O.ptr(T), O.ptr(P), O.ptr(Pn), C.c_float(maxd), C.c_float(mind),
                                  C.c_float(0.5), C.byref(px), C.byref(py), C.byref(pxr), C.byref(lvl), C.byref(vc))
    return ok, px.value, py.value, pxr.value, lvl.value, vc.value


def test_is_in_frustum_kat(oracle_mod):
    """Frame::isInFrustum(pMP, 0.5) (Frame.cc:445-501) + MapPoint::PredictScale (MapPoint.cc:
    402-417) on hand-built cases: each rejection branch, and the projection / level / view
    cosine of an accepted point against float64 arithmetic."""
    from coeb_front import synth
    O = oracle_mod
    ex = O.Extractor()
    cam = O.camera(ex, 640, 480, synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
    T = np.eye(4, dtype=np.float32)
    T[:3, 3] = (0.01, -0.02, 0.05)
    P = np.array([0.1, -0.05, 2.0], np.float32)
    Oc = -T[:3, :3].T @ T[:3, 3]
    d = np.linalg.norm(P.astype(np.float64) - Oc)
    Pn = (P - Oc) / d
    ok, u, v, ur, lvl, vc = _frustum(O, cam, T, P, Pn, d * 1.3, d * 1.3 / 3.58)
    Pc = P.astype(np.float64) + T[:3, 3]
    assert ok == 1
    assert abs(u - (synth.TUM_FX * Pc[0] / Pc[2] + synth.TUM_CX)) < 1e-3
    assert abs(v - (synth.TUM_FY * Pc[1] / Pc[2] + synth.TUM_CY)) < 1e-3
    assert abs(ur - (u - synth.TUM_BF / Pc[2])) < 1e-3
    assert lvl == math.ceil(math.log(1.3) / math.log(1.2)) == 2
    assert abs(vc - 1.0) < 1e-6
    assert _frustum(O, cam, T, P, Pn, d * 1.3 * 1.2 ** 6, d)[4] == 7          # clamped to the pyramid
    assert _frustum(O, cam, T, P, Pn, d * 0.9, d * 0.5)[4] == 0                # ratio < 1 -> level 0
    assert _frustum(O, cam, T, P * np.float32(-1), -Pn, d * 1.3, d * 0.5)[0] == 0    # behind the camera
    assert _frustum(O, cam, T, np.float32([5, 0, 2]), Pn, 10, 0.1)[0] == 0           # outside the image
    side = np.cross(Pn, [0, 1, 0]).astype(np.float32)
    side /= np.linalg.norm(side)
    assert _frustum(O, cam, T, P, side, d * 1.3, d * 0.5)[0] == 0                    # view angle > 60 deg
    tilt = (np.cos(np.radians(55)) * Pn + np.sin(np.radians(55)) * side).astype(np.float32)
    assert _frustum(O, cam, T, P, tilt, d * 1.3, d * 0.5)[0] == 1                    # 55 deg still seen
    assert _frustum(O, cam, T, P, Pn, d / 1.25, d / 4)[0] == 0                       # beyond 1.2 * maxd
    assert _frustum(O, cam, T, P, Pn, d * 3, d * 1.3)[0] == 0                        # inside 0.8 * mind


def test_oracle_track_chain_properties(oracle_mod):
    """The configs[4] loop on the oracle (track_frame: motion model + TrackLocalMap) over a
    plain synthetic sequence: every frame tracked, the local map contributes matches, the
    second optimisation keeps more inliers than the first, and a 180-degree prediction loses
    the frame (state 0) without disturbing the next one."""
    from coeb_front import synth
    O = oracle_mod
    ex = O.Extractor()
    isg = np.array(ex.p.inv_sigma2[:8], np.float32)
    F, stride = 6, 1256
    fr = synth.make_frames(640, 480, F, seed=4242)
    depth = synth.make_depth(640, 480)
    cam = O.camera(ex, 640, 480, synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
    Tcw = np.stack([synth.motion_pose()] * F)
    Tcw[3] = synth.rotated_pose(180.0, axis=1, t=(0, 0, 0))
    ext = [ex.extract(f) for f in fr]
    mfs = [O.mapframe_from_extraction(e["kps"], e["desc"], depth, synth.TUM_FX, synth.TUM_FY, synth.TUM_CX,
                                      synth.TUM_CY, synth.TUM_BF) for e in ext]
    res = [None]
    for f in range(1, F):
        ur, _ = O.stereo_from_rgbd(ext[f]["kps"], depth, synth.TUM_BF)
        res.append(O.track_frame(cam, isg, ext[f], ur, mfs[f - 1], mfs[f - 2] if f >= 2 else None, Tcw[f],
                                 res[f - 1]["T1"] if f >= 2 else np.eye(4, dtype=np.float32), stride,
                                 fx=synth.TUM_FX, fy=synth.TUM_FY, cx=synth.TUM_CX, cy=synth.TUM_CY, bf=synth.TUM_BF))
    assert [r["state"] for r in res[1:]] == [2, 2, 0, 2, 2]
    for f in (1, 2, 4, 5):
        r = res[f]
        lm = r["local_map"]
        assert lm["n_in_view"] == int(lm["in_view"].sum()) > 0
        assert r["nlocal"] > 0 and r["ninliers"] > r["nin1"]
        # local matches land on keypoints without a kept motion-model MapPoint (Observations() > 0)
        kept = (r["match"] >= 0) & (r["outlier1"] == 0)
        assert not ((r["local_match"] >= 0) & kept).any()
        # KF1 points the motion model matched are not in the local map (mnLastFrameSeen)
        assert not lm["in_view"][stride + r["match"][r["match"] >= 0]].any()
        assert np.all(lm["level"][lm["in_view"] > 0] < 8)
    assert res[1]["local_map"]["in_view"][:stride].sum() == 0          # frame 1 has no KeyFrame f-2
    assert res[3]["nlocal"] == 0 and res[3]["ninliers"] == 0
