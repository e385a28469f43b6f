"""HIP path (through the C-ABI) vs the CPU oracle, bit-exact (MI355X only).

Tolerances (BASELINE.json north_star): keypoint coordinates/octave/size/response and the
256-bit descriptors bit-exact; angles within 1e-4 degrees -- and this build also asserts
they are bit-identical (descriptors depend on the angle bits through sincosf).
"""
import os

import numpy as np
import pytest

from coeb_front import KEYPOINT_DTYPE, synth

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ANGLE_TOL = 1e-4


def assert_same(kps, desc, ref_kps, ref_desc, tag=""):
    assert len(kps) == len(ref_kps), (tag, len(kps), len(ref_kps))
    for f in KEYPOINT_DTYPE.names:
        if f == "angle":
            assert np.all(np.abs(kps[f] - ref_kps[f]) <= ANGLE_TOL), tag
        bad = np.nonzero(kps[f] != ref_kps[f])[0]
        assert len(bad) == 0, (tag, f, len(bad), kps[bad[:3]], ref_kps[bad[:3]])
    if len(kps):
        assert np.array_equal(desc, ref_desc), (tag, int((desc != ref_desc).any(axis=1).sum()))


def run_both(ctx, ex, gray, boxes=None, tm=None, blur=None, tag=""):
    r = ex.extract(gray, boxes, tm, blur)
    k, d = ctx.extract(gray, boxes, tm, blur)
    assert_same(k, d, r["kps"], r["desc"], tag)
    return k, d


@pytest.fixture(scope="module")
def ex(oracle_mod):
    return oracle_mod.Extractor()


def test_golden_extract(ctx):
    g = np.load(os.path.join(HERE, "golden", "extract_A.npz"))
    for name in ("plain", "dyn", "area"):
        args = () if name == "plain" else (g[name + "_boxes"], g[name + "_tm"], g[name + "_blur"])
        k, d = ctx.extract(g["frame"], *args)
        assert_same(k, d, g[name + "_kps"], g[name + "_desc"], name)


@pytest.mark.parametrize("seed", [1000, 1001, 1002, 7])
def test_extract_A_frames(ctx, ex, seed):
    fr = synth.make_frames(640, 480, 3, seed=seed)
    for i in range(3):
        run_both(ctx, ex, fr[i], tag="seed%d f%d" % (seed, i))


def test_extract_B_1280x960(ctx, oracle_mod):
    ex2 = oracle_mod.Extractor(2000, 1.2, 8, 20, 7)
    from coeb_front import Context
    c2 = Context(2000, 1.2, 8, 20, 7, max_width=1280, max_height=960)
    try:
        fr = synth.make_frames(1280, 960, 1, seed=2000)
        run_both(c2, ex2, fr[0], tag="B")
        b, t, bl = synth.dynamic_inputs(1280, 960)
        run_both(c2, ex2, fr[0], b, t, bl, tag="B dyn")
    finally:
        c2.close()


def test_fast_general_slab_layout_matches_oracle(ctx, ex, monkeypatch):
    """k_fast keeps the ROI pixels and the corner strengths M in one 96-byte slab row when every
    ROI is at most 46 wide (the 640x480 plans) and in a 72-byte slab plus a compact M slab
    otherwise (320x240: its top level has one 57-px cell).  COEB_FAST_RB=72 forces the general
    layout on the 640x480 plan too; both must equal the oracle, including a noise image whose
    cells overflow the corner list (whole-window NMS)."""
    monkeypatch.setenv("COEB_FAST_RB", "72")
    for seed in (1000, 7):
        run_both(ctx, ex, synth.make_frames(640, 480, 1, seed=seed)[0], tag="rb72 %d" % seed)
    rng = np.random.default_rng(5)
    run_both(ctx, ex, rng.integers(0, 256, (480, 640), dtype=np.uint8), tag="rb72 noise")
    monkeypatch.delenv("COEB_FAST_RB")
    run_both(ctx, ex, rng.integers(0, 256, (480, 640), dtype=np.uint8), tag="rb96 noise")


@pytest.mark.parametrize("w,h", [(641, 479), (320, 240), (800, 600), (1024, 768), (720, 405)])
def test_extract_ragged_sizes(ctx, ex, w, h):
    fr = synth.make_frames(w, h, 1, seed=w * 7 + h)
    run_both(ctx, ex, fr[0], tag="%dx%d" % (w, h))


@pytest.mark.parametrize("pyr_form", ["rows", "bytes"])
@pytest.mark.parametrize("w,h", [(640, 480), (641, 479), (533, 400), (1280, 960), (720, 405)])
def test_blur_pyramid_matches_oracle(ctx, ex, oracle_mod, w, h, pyr_form, monkeypatch):
    """k_blur's whole blurred pyramid (not only the pixels rBRIEF samples) equals the oracle's
    GaussianBlur of each oracle pyramid level (ORBextractor.cc:1317-1318), every pixel including
    the REFLECT_101 borders and the partial 64-column strips of ragged widths.  Both pyramid
    kernels: k_pyr_rows (default where rows are 4-byte aligned) and k_pyr_level's byte form
    (COEB_PYR_BYTES=1; the only form for odd-pitch inputs such as 641x479's level 0).  The raw
    pyramid levels are compared too."""
    if pyr_form == "bytes":
        monkeypatch.setenv("COEB_PYR_BYTES", "1")
    from coeb_front import Context
    c2 = ctx if (w, h) != (1280, 960) else Context(2000, 1.2, 8, 20, 7, max_width=w, max_height=h)
    ex2 = ex if c2 is ctx else oracle_mod.Extractor(2000, 1.2, 8, 20, 7)
    try:
        gray = synth.make_frames(w, h, 1, seed=w + 3 * h)[0]
        r = ex2.extract(gray, debug=True)
        c2.extract(gray)
        blur = c2.debug_read("blur")
        pyr = c2.debug_read("pyr")
        off = poff = 0
        for l, (lw, lh) in enumerate(ex2.level_sizes(w, h)):
            lvl = gray if l == 0 else r["pyramid"][r["level_off"][l]:r["level_off"][l] + lw * lh].reshape(lh, lw)
            if l > 0:
                pp = (lw + 63) // 64 * 64
                gotp = pyr[poff:poff + pp * lh].reshape(lh, pp)[:, :lw]
                badp = np.argwhere(gotp != lvl)
                assert len(badp) == 0, ("pyramid level", l, len(badp), badp[:4].tolist())
                poff = (poff + pp * lh + 255) // 256 * 256
            ref = oracle_mod.gaussian_blur7(lvl)
            pitch = (lw + 63) // 64 * 64
            got = blur[off:off + pitch * lh].reshape(lh, pitch)[:, :lw]
            bad = np.argwhere(got != ref)
            assert len(bad) == 0, ("level", l, len(bad), bad[:4].tolist())
            off = (off + pitch * lh + 255) // 256 * 256
    finally:
        if c2 is not ctx:
            c2.close()


@pytest.mark.parametrize("nfeat,scale,nlev", [(500, 1.2, 8), (2000, 1.2, 8), (1000, 1.3, 6), (1000, 1.2, 4),
                                              (1000, 1.1, 10)])
def test_extract_params(oracle_mod, nfeat, scale, nlev):
    """nlevels = 10 exercises CheckMovingKeyPoints_finall's hard-coded 8-level loop."""
    from coeb_front import Context
    ex2 = oracle_mod.Extractor(nfeat, scale, nlev, 20, 7)
    c2 = Context(nfeat, scale, nlev, 20, 7, max_width=640, max_height=480)
    try:
        fr = synth.make_frames(640, 480, 1, seed=nfeat + nlev)
        run_both(c2, ex2, fr[0], tag="params")
        b, t, bl = synth.dynamic_inputs(640, 480)
        run_both(c2, ex2, fr[0], b, t, bl, tag="params dyn")
    finally:
        c2.close()


@pytest.mark.parametrize("scale,nlev", [(2.0, 5), (4.0, 3)])
def test_extract_params_reference_ub_rejected(oracle_mod, scale, nlev):
    """A pyramid level narrower than one 30-px FAST cell gives nCols = 0 and a division by zero
    in the reference (ORBextractor.cc:806-808, UB): 640x480 at scale 2.0 / 5 levels has a 40x30
    level 4.  The oracle refuses it (rc -1 from oc_extract) and the HIP path returns COEB_EINVAL
    with a message instead of launching."""
    from coeb_front import CoebError, Context
    fr = synth.make_frames(640, 480, 1, seed=3)[0]
    with pytest.raises(RuntimeError, match=r"oc_extract rc=-"):
        oracle_mod.Extractor(1000, scale, nlev, 20, 7).extract(fr)
    c2 = Context(1000, scale, nlev, 20, 7, max_width=640, max_height=480)
    try:
        with pytest.raises(CoebError, match=r"rc=-22: pyramid level too small"):
            c2.extract(fr)
    finally:
        c2.close()


def test_extract_edge_images(ctx, ex):
    # constant: no corners at all; near-constant: only minThFAST fallback corners
    run_both(ctx, ex, np.full((480, 640), 128, np.uint8), tag="const")
    rng = np.random.default_rng(5)
    run_both(ctx, ex, np.clip(128 + rng.integers(-5, 6, (480, 640)), 0, 255).astype(np.uint8), tag="low")
    # high texture: thousands of candidates per level (octree final phase, size ties)
    run_both(ctx, ex, rng.integers(0, 256, (480, 640), dtype=np.uint8), tag="noise")
    chk = ((np.indices((480, 640)).sum(axis=0) // 3) % 2 * 255).astype(np.uint8)
    run_both(ctx, ex, chk, tag="checker")
    k, d = ctx.extract(np.zeros((0, 0), np.uint8))
    assert len(k) == 0 and d is None


def test_extract_dynamic_masks(ctx, ex):
    fr = synth.make_frames(640, 480, 1, seed=1234)[0]
    b, t, bl = synth.dynamic_inputs(640, 480, seed=3)
    run_both(ctx, ex, fr, b, t, bl, tag="dyn")
    run_both(ctx, ex, fr, b, t, None, tag="no blur flags (missing -> 0)")
    run_both(ctx, ex, fr, b, t[:0], np.array([1, 1], np.int32), tag="no T_M")
    b2, t2, bl2 = synth.dynamic_inputs(640, 480, seed=4, area_flag=True)
    run_both(ctx, ex, fr, b2, t2, bl2, tag="area")
    # fractional boxes: Rect(int(x), int(y), int(w), int(h)) vs fill loop (int)xmin..(int)xmax
    b3 = np.array([[100.7, 50.2, 300.4, 420.9], [0.0, 0.0, 639.0, 479.0]], np.float32)
    t3 = np.array([[150.5, 60.5], [299.9, 419.9], [10, 10]], np.float32)
    run_both(ctx, ex, fr, b3, t3, np.array([1, 0], np.int32), tag="fractional")


def test_blur_flags(ctx, oracle_mod):
    from coeb_front import lib
    import ctypes as C
    fr = synth.make_frames(640, 480, 1, seed=9)[0]
    sm = fr.copy()
    sm[100:300, 200:320] = 90           # flat region -> blurred -> flag 1
    boxes = np.array([[200, 100, 320, 300], [10.5, 20.5, 200.2, 400.7], [630, 470, 640, 480], [0, 0, 1, 1],
                      [-5, 0, 10, 10]], np.float32)
    ref, _ = oracle_mod.blur_flags(sm, boxes)
    out = np.zeros(len(boxes), np.int32)
    ctx.check(lib().coeb_blur_flags(ctx.h, sm.ctypes.data_as(C.c_void_p), 640, 480, 640,
                                    boxes.ctypes.data_as(C.c_void_p), len(boxes), out.ctypes.data_as(C.c_void_p)))
    assert np.array_equal(out, ref) and ref[0] == 1


@pytest.mark.parametrize("channels,mbrgb", [(3, True), (3, False), (4, True), (4, False), (1, True)])
def test_rgbd_preprocess_formats(ctx, oracle_mod, channels, mbrgb):
    """Tracking::GrabImageRGBD (Tracking.cc:212-228): RGB / BGR / RGBA / BGRA / gray images, with
    a ragged row stride, against the oracle; 16UC1 depth scaled, 32FC1 depth scaled or (factor 1)
    passed through bit-for-bit."""
    import coeb_front
    rng = np.random.default_rng(channels * 10 + mbrgb)
    h, w = 121, 203
    shape = (h, w) if channels == 1 else (h, w, channels)
    img = rng.integers(0, 256, shape, dtype=np.uint8)
    d16 = rng.integers(0, 65535, (h, w), dtype=np.uint16)
    gray, dep = coeb_front.GrabImageRGBD(ctx, img, d16, mbrgb, np.float32(1 / 5000.0))
    assert np.array_equal(gray, oracle_mod.image_to_gray(img, 1 if mbrgb else 0))
    assert np.array_equal(dep, oracle_mod.depth_to_float(d16, np.float32(1 / 5000.0)))
    assert np.array_equal(dep, d16.astype(np.float32) * np.float32(1 / 5000.0))
    d32 = (rng.random((h, w)) * 8).astype(np.float32)
    d32[0, :4] = [np.nan, np.inf, -0.0, 0.0]
    for factor in (1.0, 1.0 + 5e-6, 0.5, 1 / 5000.0):
        _, dep = coeb_front.GrabImageRGBD(ctx, img, d32, mbrgb, np.float32(factor))
        ref = oracle_mod.depth_to_float(d32, np.float32(factor))
        assert np.array_equal(dep.view(np.uint32), ref.view(np.uint32)), factor
        if abs(np.float32(factor) - 1) <= 1e-5:
            assert np.array_equal(dep.view(np.uint32), d32.view(np.uint32))     # :227 passthrough
    # a sub-view with a row stride larger than the row (ctypes sees the parent's pitch)
    big = rng.integers(0, 256, (h, w + 9) + (() if channels == 1 else (channels,)), dtype=np.uint8)
    view = big[:, :w]
    from coeb_front import lib
    import ctypes as C
    out = np.zeros((h, w), np.uint8)
    ctx.check(lib().coeb_rgbd_preprocess(ctx.h, big.ctypes.data_as(C.c_void_p), big.strides[0], channels,
                                         1 if mbrgb else 0, None, 0, 0, C.c_float(1.0), w, h,
                                         out.ctypes.data_as(C.c_void_p), None))
    assert np.array_equal(out, oracle_mod.image_to_gray(np.ascontiguousarray(view), 1 if mbrgb else 0))


def test_rgbd_preprocess_rejects_bad_arguments(ctx):
    from coeb_front import CoebError, lib
    import ctypes as C
    img = np.zeros((8, 8, 2), np.uint8)
    out = np.zeros((8, 8), np.uint8)
    for ch in (0, 2, 5):
        rc = lib().coeb_rgbd_preprocess(ctx.h, img.ctypes.data_as(C.c_void_p), 16, ch, 1, None, 0, 0,
                                        C.c_float(1.0), 8, 8, out.ctypes.data_as(C.c_void_p), None)
        assert rc == -22
    d = np.zeros((8, 8), np.uint16)
    rc = lib().coeb_rgbd_preprocess(ctx.h, None, 0, 3, 1, d.ctypes.data_as(C.c_void_p), 16, 7, C.c_float(1.0), 8, 8,
                                    None, out.ctypes.data_as(C.c_void_p))
    assert rc == -22
    assert CoebError


def test_rgbd_preprocess_and_stereo(ctx, oracle_mod):
    import coeb_front
    from coeb_front import lib
    import ctypes as C
    rng = np.random.default_rng(3)
    rgb = rng.integers(0, 256, (480, 640, 3), dtype=np.uint8)
    d16 = rng.integers(0, 6000, (480, 640), dtype=np.uint16)
    gray, dep = coeb_front.GrabImageRGBD(ctx, rgb, d16, True, np.float32(1 / 5000.0))
    assert np.array_equal(gray, oracle_mod.rgb2gray(rgb, 1))
    assert np.array_equal(dep, d16.astype(np.float32) * np.float32(1 / 5000.0))
    k, d = ctx.extract(gray)
    ur_ref, dep_ref = oracle_mod.stereo_from_rgbd(k, dep, synth.TUM_BF)
    ur = np.zeros(len(k), np.float32)
    dd = np.zeros(len(k), np.float32)
    ctx.check(lib().coeb_stereo_from_rgbd(ctx.h, k.ctypes.data_as(C.c_void_p), len(k), dep.ctypes.data_as(C.c_void_p),
                                          640, 480, 640, C.c_float(synth.TUM_BF), ur.ctypes.data_as(C.c_void_p),
                                          dd.ctypes.data_as(C.c_void_p)))
    assert np.array_equal(ur, ur_ref) and np.array_equal(dd, dep_ref)


# ------------------------------------------------------------------ matcher
def match_both(ctx, oracle_mod, ex, cur_k, cur_d, cur_ur, last, Tc, Tl, th=15.0, bmono=False, check_ori=True):
    import coeb_front
    cam_o = oracle_mod.camera(ex, 640, 480, synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
    nm_ref, m_ref = oracle_mod.search_by_projection(cam_o, cur_k, cur_d, cur_ur, last, Tc, Tl, th, bmono, check_ori)
    cam = coeb_front.make_camera(synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF, 640, 480)
    cur = coeb_front.Frame(cur_k, cur_d, cur_ur, Tcw=Tc)
    lf = coeb_front.Frame(last["keys_un"], last["mp_desc"], Tcw=Tl, outlier=last["outlier"],
                          map_points=dict(world_pos=last["xw"], descriptor=last["mp_desc"],
                                          observations=last["mp_nobs"], valid=last["has_mp"]))
    m = coeb_front.ORBmatcher(0.9, check_ori, ctx=ctx)
    nm = m.SearchByProjection(cur, lf, th, bmono, cam)
    assert nm == nm_ref and np.array_equal(cur.mvpMapPoints, m_ref), (nm, nm_ref)
    return nm


def test_golden_match(ctx, oracle_mod, ex):
    g = np.load(os.path.join(HERE, "golden", "match_A.npz"))
    last = {k[5:]: g[k] for k in g.files if k.startswith("last_")}
    nm = match_both(ctx, oracle_mod, ex, g["cur_kps"], g["cur_desc"], g["cur_ur"], last, g["Tcw_cur"], g["Tcw_last"])
    assert nm == int(g["nmatches"])


@pytest.fixture(scope="module")
def pair(oracle_mod, ex):
    fr = synth.make_frames(640, 480, 2, seed=77)
    r0, r1 = ex.extract(fr[0]), ex.extract(fr[1])
    depth = synth.make_depth(640, 480)
    last = oracle_mod.mapframe_from_extraction(r0["kps"], r0["desc"], depth, synth.TUM_FX, synth.TUM_FY,
                                               synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
    ur1, _ = oracle_mod.stereo_from_rgbd(r1["kps"], depth, synth.TUM_BF)
    return r1, ur1, last


def test_match_variants(ctx, oracle_mod, ex, pair):
    r1, ur1, last = pair
    Tc, Tl = synth.motion_pose(), np.eye(4, dtype=np.float32)
    rng = np.random.default_rng(11)
    n = len(last["has_mp"])
    v = dict(last)
    v["mp_nobs"] = np.where(rng.random(n) < 0.3, 0, 2).astype(np.int32)   # claim-overwrite path
    match_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], ur1, v, Tc, Tl)
    v = dict(last)
    v["outlier"] = (rng.random(n) < 0.2).astype(np.uint8)
    v["has_mp"] = (last["has_mp"] & (rng.random(n) < 0.8)).astype(np.uint8)
    match_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], ur1, v, Tc, Tl)
    match_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], ur1, last, Tc, Tl, check_ori=False)
    match_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], ur1, last, Tc, Tl, bmono=True)
    match_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], ur1, last, Tc, Tl, th=30.0)
    match_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], np.full(len(ur1), -1, np.float32), last, Tc, Tl)
    for tz in (0.5, -0.5):            # bForward / bBackward level windows
        T = Tc.copy()
        T[2, 3] = tz
        match_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], ur1, last, T, Tl)
    # empty frames
    e = {k: val[:0] for k, val in last.items()}
    assert match_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], ur1, e, Tc, Tl) == 0


def test_match_paths_agree(ctx, oracle_mod, ex, pair, monkeypatch):
    """The parallel fixpoint claim resolution and the literal sequential loop (forced with
    COEB_MATCH_SEQUENTIAL) both equal the oracle."""
    r1, ur1, last = pair
    Tc, Tl = synth.motion_pose(), np.eye(4, dtype=np.float32)
    rng = np.random.default_rng(12)
    v = dict(last)
    v["mp_nobs"] = np.where(rng.random(len(last["has_mp"])) < 0.5, 0, 2).astype(np.int32)
    for seq in (False, True):
        if seq:
            monkeypatch.setenv("COEB_MATCH_SEQUENTIAL", "1")
        match_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], ur1, v, Tc, Tl)
        match_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], ur1, last, Tc, Tl, th=30.0)
    monkeypatch.delenv("COEB_MATCH_SEQUENTIAL")


def test_match_repetitive_texture(ctx, oracle_mod, ex):
    """Repetitive structure -> many near-identical descriptors per window: exercises long
    candidate lists (and the sequential fallback when a list overflows)."""
    yy, xx = np.indices((480, 640))
    base = (((yy // 12) + (xx // 12)) % 2 * 200 + 30).astype(np.int16)
    rng = np.random.default_rng(8)
    f0 = np.clip(base + rng.integers(-6, 7, base.shape), 0, 255).astype(np.uint8)
    f1 = np.clip(np.roll(base, (1, 2), axis=(0, 1)) + rng.integers(-6, 7, base.shape), 0, 255).astype(np.uint8)
    r0, r1 = ex.extract(f0), ex.extract(f1)
    depth = synth.make_depth(640, 480)
    last = oracle_mod.mapframe_from_extraction(r0["kps"], r0["desc"], depth, synth.TUM_FX, synth.TUM_FY,
                                               synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
    ur1, _ = oracle_mod.stereo_from_rgbd(r1["kps"], depth, synth.TUM_BF)
    for th in (15.0, 30.0, 60.0):
        match_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], ur1, last, synth.motion_pose(),
                   np.eye(4, dtype=np.float32), th=th)


# ------------------------------------------------------------------ batch (device-resident) path
def test_batch_pipeline_matches_oracle(oracle_mod, ex):
    from coeb_front.pipeline import BatchPipeline
    F = 6
    fr = synth.make_frames(640, 480, F, seed=4242)
    Tcw = np.stack([synth.motion_pose()] * F)
    bp = BatchPipeline(640, 480, F)
    try:
        dyn = [synth.dynamic_inputs(640, 480, seed=f) if f % 2 else (None, None, None) for f in range(F)]
        bp.load(fr, Tcw=Tcw, dyn=dyn)
        bp.run()
        bp.synchronize()
        out, matches, nms = bp.results()
        depth = synth.make_depth(640, 480)
        cam_o = oracle_mod.camera(ex, 640, 480, synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
        prev = None
        for f in range(F):
            b, t, bl = dyn[f]
            r = ex.extract(fr[f], b, t, bl)
            assert_same(out[f][0], out[f][1], r["kps"], r["desc"], "batch f%d" % f)
            if prev is not None:
                last = oracle_mod.mapframe_from_extraction(prev["kps"], prev["desc"], depth, synth.TUM_FX,
                                                           synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
                ur, _ = oracle_mod.stereo_from_rgbd(r["kps"], depth, synth.TUM_BF)
                I4 = np.eye(4, dtype=np.float32)
                nm, m = oracle_mod.search_by_projection(cam_o, r["kps"], r["desc"], ur, last, Tcw[f], I4, 15.0)
                if nm < 20:                                      # Tracking.cc:954-958
                    nm, m = oracle_mod.search_by_projection(cam_o, r["kps"], r["desc"], ur, last, Tcw[f], I4, 30.0)
                assert nms[f] == nm and np.array_equal(matches[f], m), (f, nms[f], nm)
            prev = r
        # idempotence: a second run gives identical outputs
        bp.run()
        bp.synchronize()
        out2, matches2, nms2 = bp.results()
        assert all(np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) for a, b in zip(out, out2))
        assert nms == nms2
        # host-pose entry point (coeb_match_batch_device) == device-pose one
        bp.ctx.match_batch_device(bp.depth.ptr, F, 640, 480, bp.cam, Tcw)
        bp.synchronize()
        _, matches3, nms3 = bp.results()
        assert nms3 == nms and all(np.array_equal(a, b) for a, b in zip(matches[1:], matches3[1:]))
    finally:
        bp.close()


@pytest.mark.parametrize("mode", ["default", "sequential", "nosplit"])
def test_batch_small_split_lists_matches_oracle(oracle_mod, ex, monkeypatch, mode):
    """Few pairs per launch (P < 128): the candidate lists come from k_match_lists split over
    several workgroups per pair, and k_match starts at the claims without the current frame staged
    in LDS.  Its late paths -- list overflow on repetitive texture (sequential fallback), the
    literal sequential pass (COEB_MATCH_SEQUENTIAL=1) and the 2*th retry of a frame whose
    prediction is 180 degrees off -- must equal the oracle frame by frame; COEB_MATCH_SPLIT=0
    runs the unsplit kernel on the same batch."""
    from coeb_front.pipeline import BatchPipeline
    if mode == "sequential":
        monkeypatch.setenv("COEB_MATCH_SEQUENTIAL", "1")
    elif mode == "nosplit":
        monkeypatch.setenv("COEB_MATCH_SPLIT", "0")
    F = 7
    yy, xx = np.indices((480, 640))
    base = (((yy // 12) + (xx // 12)) % 2 * 200 + 30).astype(np.int16)
    rng = np.random.default_rng(31)
    fr = np.stack([np.clip(np.roll(base, (f, 2 * f), axis=(0, 1)) + rng.integers(-6, 7, base.shape), 0, 255)
                   for f in range(4)] + list(synth.make_frames(640, 480, F - 4, seed=313))).astype(np.uint8)
    Tcw = np.stack([synth.motion_pose()] * F)
    Tcw[5] = synth.rotated_pose(180.0, axis=1, t=(0, 0, 0))          # < 20 matches: the 2*th retry runs
    depth = synth.make_depth(640, 480)
    cam_o = oracle_mod.camera(ex, 640, 480, synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
    I4 = np.eye(4, dtype=np.float32)
    ref = [ex.extract(f) for f in fr]
    bp = BatchPipeline(640, 480, F)
    try:
        bp.load(fr, Tcw=Tcw)
        for th in (15.0, 60.0):
            bp.run(th=th)
            bp.synchronize()
            out, matches, nms = bp.results()
            for f in range(F):
                assert_same(out[f][0], out[f][1], ref[f]["kps"], ref[f]["desc"], "split f%d" % f)
                if f == 0:
                    continue
                last = oracle_mod.mapframe_from_extraction(ref[f - 1]["kps"], ref[f - 1]["desc"], depth, synth.TUM_FX,
                                                           synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
                ur, _ = oracle_mod.stereo_from_rgbd(ref[f]["kps"], depth, synth.TUM_BF)
                nm, m = oracle_mod.search_by_projection(cam_o, ref[f]["kps"], ref[f]["desc"], ur, last, Tcw[f], I4, th)
                if nm < 20:                                          # Tracking.cc:954-958
                    nm, m = oracle_mod.search_by_projection(cam_o, ref[f]["kps"], ref[f]["desc"], ur, last, Tcw[f],
                                                            I4, 2 * th)
                assert nms[f] == nm and np.array_equal(matches[f], m), (mode, th, f, nms[f], nm)
            assert nms[5] < 20
    finally:
        bp.close()


def test_batch_track_pose_matches_oracle(oracle_mod, ex):
    """BASELINE configs[4] slice on the device batch: extract + SearchByProjection + the
    TrackWithMotionModel PoseOptimization (Tracking.cc:947-964) for every pair, against the
    oracle run frame by frame (extract -> search with retry -> pose_optimization).  Frame 3
    gets a prediction 180 degrees off: < 20 matches, so it must stay untracked (pose = the
    prediction, 0 inliers)."""
    from coeb_front.pipeline import BatchPipeline
    F = 6
    fr = synth.make_frames(640, 480, F, seed=777)
    Tcw = np.stack([synth.motion_pose()] * F)
    Tcw[3] = synth.rotated_pose(180.0, axis=1, t=(0, 0, 0))
    bp = BatchPipeline(640, 480, F)
    try:
        bp.load(fr, Tcw=Tcw)
        bp.run(pose=True)
        bp.synchronize()
        out, matches, nms = bp.results()
        T_dev, nin_dev, outl_dev = bp.pose_results()
        depth = synth.make_depth(640, 480)
        cam_o = oracle_mod.camera(ex, 640, 480, synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
        isg = np.array(bp.ctx.tables().inv_sigma2[:8], np.float32)
        I4 = np.eye(4, dtype=np.float32)
        prev = ex.extract(fr[0])
        tracked = 0
        for f in range(1, F):
            r = ex.extract(fr[f])
            last = oracle_mod.mapframe_from_extraction(prev["kps"], prev["desc"], depth, synth.TUM_FX, synth.TUM_FY,
                                                       synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
            ur, _ = oracle_mod.stereo_from_rgbd(r["kps"], depth, synth.TUM_BF)
            nm, m = oracle_mod.search_by_projection(cam_o, r["kps"], r["desc"], ur, last, Tcw[f], I4, 15.0)
            if nm < 20:
                nm, m = oracle_mod.search_by_projection(cam_o, r["kps"], r["desc"], ur, last, Tcw[f], I4, 30.0)
            assert nms[f] == nm and np.array_equal(matches[f], m), f
            if nm < 20:                                          # Tracking.cc:954-958: not tracked
                assert nin_dev[f] == 0 and np.array_equal(T_dev[f].view(np.uint32), Tcw[f].view(np.uint32)), f
            else:
                has = (m >= 0).astype(np.uint8)
                xw = np.zeros((len(m), 3), np.float32)
                xw[m >= 0] = last["xw"][m[m >= 0]]
                nin, T_ref, o_ref = oracle_mod.pose_optimization(r["kps"], has, xw, ur, isg, synth.TUM_FX, synth.TUM_FY,
                                                                 synth.TUM_CX, synth.TUM_CY, synth.TUM_BF, Tcw[f])
                assert nin_dev[f] == nin and nin > 0, (f, nin_dev[f], nin)
                assert np.array_equal(T_dev[f].view(np.uint32), T_ref.view(np.uint32)), f
                assert np.array_equal(outl_dev[f][has > 0], o_ref[has > 0]), f
                tracked += 1
            prev = r
        assert tracked == F - 2 and nin_dev[3] == 0
        # pipelined: step k's k_pose (own stream) overlaps step k+1's extraction and matching;
        # three back-to-back steps must leave exactly the single-step results
        for _ in range(3):
            bp.run(pose=True)
        T2, nin2, outl2 = bp.pose_results()
        assert nin2 == nin_dev and np.array_equal(T2[1:].view(np.uint32), T_dev[1:].view(np.uint32))
        assert all(np.array_equal(a, b) for a, b in zip(outl2[1:], outl_dev[1:]))
    finally:
        bp.close()


def test_batch_B_full_size_properties(oracle_mod):
    """Config B at full size: 1280x960, 2000 kp, batch of 16 -- every frame's keypoints,
    descriptors and SearchByProjection result (with the 2*th retry) equal to the oracle's, plus
    the size-independent properties."""
    from coeb_front.pipeline import BatchPipeline
    F = 16
    W, H = 1280, 960
    fr = synth.make_frames(W, H, F, seed=99)
    Tcw = np.stack([synth.motion_pose()] * F)
    bp = BatchPipeline(W, H, F, nfeatures=2000)
    try:
        bp.load(fr, Tcw=Tcw)
        bp.run()
        bp.synchronize()
        out, matches, nms = bp.results()
        ex2 = oracle_mod.Extractor(2000, 1.2, 8, 20, 7)
        depth = synth.make_depth(W, H)
        cam_o = oracle_mod.camera(ex2, W, H, synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
        I4 = np.eye(4, dtype=np.float32)
        prev = None
        for f in range(F):
            r = ex2.extract(fr[f])
            assert_same(out[f][0], out[f][1], r["kps"], r["desc"], "B batch f%d" % f)
            if prev is not None:
                last = oracle_mod.mapframe_from_extraction(prev["kps"], prev["desc"], depth, synth.TUM_FX, synth.TUM_FY,
                                                           synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
                ur, _ = oracle_mod.stereo_from_rgbd(r["kps"], depth, synth.TUM_BF)
                nm, m = oracle_mod.search_by_projection(cam_o, r["kps"], r["desc"], ur, last, Tcw[f], I4, 15.0)
                if nm < 20:                                      # Tracking.cc:954-958
                    nm, m = oracle_mod.search_by_projection(cam_o, r["kps"], r["desc"], ur, last, Tcw[f], I4, 30.0)
                assert nms[f] == nm and np.array_equal(matches[f], m), (f, nms[f], nm)
            prev = r
        for f in range(F):
            k = out[f][0]
            assert 0 < len(k) <= 2000 + 8 * 8
            assert (k["x"] >= 0).all() and (k["x"] < 1280).all() and (k["y"] >= 0).all() and (k["y"] < 960).all()
            assert set(np.unique(k["octave"])) <= set(range(8))
            assert (k["class_id"] == -1).all()
            if f:
                m = matches[f]
                assert (m >= -1).all() and (m < len(out[f - 1][0])).all()
                assert nms[f] == int((m >= 0).sum()) and nms[f] > 0.5 * len(k)
                used = m[m >= 0]
                assert len(np.unique(used)) == len(used)     # a LastFrame point matches at most once
    finally:
        bp.close()


def test_batch_streams_agree(oracle_mod, ex):
    """The batch chunked over 4 HIP streams (kernels of different chunks overlapping, several
    steps enqueued back to back) gives the same bits as the serial single-stream batch, and the
    frames on either side of each chunk boundary match the oracle."""
    from coeb_front.pipeline import BatchPipeline
    F = 65
    fr = synth.make_frames(640, 480, F, seed=777)
    bp = BatchPipeline(640, 480, F)
    try:
        bp.load(fr, Tcw=np.stack([synth.motion_pose()] * F))
        res = {}
        for ns in (1, 4, 3, 1):
            bp.ctx.set_batch_streams(ns)
            for _ in range(3):
                bp.run()
            bp.synchronize()
            res.setdefault(ns, []).append(bp.results())
        out1, m1, n1 = res[1][0]
        for ns, runs in res.items():
            for out, m, n in runs:
                assert n == n1, ns
                for f in range(F):
                    assert np.array_equal(out[f][0], out1[f][0]) and np.array_equal(out[f][1], out1[f][1]), (ns, f)
                    if f:
                        assert np.array_equal(m[f], m1[f]), (ns, f)
        depth = synth.make_depth(640, 480)
        cam_o = oracle_mod.camera(ex, 640, 480, synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
        I4 = np.eye(4, dtype=np.float32)
        for f in (16, 32, 48):       # 4-chunk boundaries: frame f is the first of its chunk
            rp, r = ex.extract(fr[f - 1]), ex.extract(fr[f])
            assert_same(out1[f][0], out1[f][1], r["kps"], r["desc"], "f%d" % f)
            last = oracle_mod.mapframe_from_extraction(rp["kps"], rp["desc"], depth, synth.TUM_FX, synth.TUM_FY,
                                                       synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
            ur, _ = oracle_mod.stereo_from_rgbd(r["kps"], depth, synth.TUM_BF)
            nm, mm = oracle_mod.search_by_projection(cam_o, r["kps"], r["desc"], ur, last, synth.motion_pose(), I4, 15.0)
            if nm < 20:
                nm, mm = oracle_mod.search_by_projection(cam_o, r["kps"], r["desc"], ur, last, synth.motion_pose(), I4,
                                                         30.0)
            assert n1[f] == nm and np.array_equal(m1[f], mm), f
    finally:
        bp.close()


@pytest.mark.parametrize("side", ["own", "shared", "eager", "off"])
def test_sharded_batch_equals_unsharded(monkeypatch, side):
    """SURVEY.md s8e partitioning: a 24-frame sequence split over 3 shards (each with its one-frame
    halo, `dist.shard_frames`), driven concurrently from 3 host threads with one context each (what
    `bench.py --gpus N` does per device; all on device 0 here), gives per-frame keypoints,
    descriptors and matches bit-identical to the unsharded batch.  "shared": the three contexts'
    extraction side work goes to one per-device side stream (COEB_SIDE_SHARED=1, bench.py config C);
    "eager": each context's side stream is created with the context (COEB_SIDE_EAGER=1, config A);
    "off": no side stream (COEB_SIDE_STREAM=0, the profiling passes' schedule)."""
    monkeypatch.setenv("COEB_SIDE_SHARED", "1" if side == "shared" else "0")
    monkeypatch.setenv("COEB_SIDE_EAGER", "1" if side == "eager" else "0")
    monkeypatch.setenv("COEB_SIDE_STREAM", "0" if side == "off" else "1")
    import threading
    from coeb_front.dist import shard_frames
    from coeb_front.pipeline import BatchPipeline
    G, world = 24, 3
    seq = synth.make_frames(640, 480, G + 1, seed=1000)
    full = BatchPipeline(640, 480, G + 1)
    try:
        full.load(seq, Tcw=np.stack([synth.motion_pose()] * (G + 1)))
        full.run()
        full.synchronize()
        ref_out, ref_m, ref_n = full.results()
    finally:
        full.close()
    got, errs = {}, []

    def rank(r):
        try:
            first, F, nm = shard_frames(G, world, r)
            fr = synth.make_frames(640, 480, F, seed=1000, first=first)
            assert np.array_equal(fr, seq[first:first + F])
            bp = BatchPipeline(640, 480, F)
            try:
                bp.load(fr, Tcw=np.stack([synth.motion_pose()] * F))
                for _ in range(2):
                    bp.run()
                bp.synchronize()
                got[r] = (first, bp.results())
            finally:
                bp.close()
        except BaseException as e:    # noqa: BLE001
            errs.append(e)
    ths = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errs, errs
    covered = []
    for r in range(world):
        first, (out, m, n) = got[r]
        for i in range(1, len(out)):
            g = first + i
            covered.append(g)
            assert np.array_equal(out[i][0], ref_out[g][0]) and np.array_equal(out[i][1], ref_out[g][1]), g
            assert n[i] == ref_n[g] and np.array_equal(m[i], ref_m[g]), g
    assert covered == list(range(1, G + 1))


@pytest.mark.parametrize("mode,shared", [("ring", True), ("slot", True), ("copyq", True), ("copyq", False)])
def test_host_stream_overlapped_equals_device_batch(mode, shared):
    """The PCIe-inclusive pipeline (HostStream: page-locked host frames in, host results out, two
    slots whose copies overlap each other's kernels) returns per-frame keypoints, descriptors and
    matches bit-identical to the device-resident batch, for several batches in flight, with the
    copies on each slot's own stream or on copy queues."""
    from coeb_front import HostBuffer
    from coeb_front.pipeline import BatchPipeline, HostStream
    F = 9
    seqs = [synth.make_frames(640, 480, F, seed=s) for s in (11, 12, 13)]
    Tcw = np.stack([synth.motion_pose()] * F)
    ref = []
    bp = BatchPipeline(640, 480, F)
    try:
        for fr in seqs:
            bp.load(fr, Tcw=Tcw)
            bp.run()
            bp.synchronize()
            ref.append(bp.results())
    finally:
        bp.close()
    hs = HostStream(640, 480, F, Tcw=Tcw, mode=mode, shared_queue=shared)
    bufs = [HostBuffer(F * 480 * 640) for _ in seqs]
    try:
        for b, fr in zip(bufs, seqs):
            b.view(np.uint8, (F, 480, 640))[:] = fr
        got = []
        for i in range(4):                      # batches 0,1,2,0 with two in flight
            hs.submit(i, bufs[i % 3])
            if i:
                hs.wait(i - 1)
                got.append(hs.results(i - 1))
        hs.wait(3)
        got.append(hs.results(3))
        # submit-only loop (device-side ordering): the last two results
        for i in range(4, 9):
            hs.submit(i, bufs[i % 3])
        hs.wait(7)
        last7 = hs.results(7)
        hs.wait(8)
        got += [last7, hs.results(8)]
        for j, (out, m, n) in enumerate(got):
            i = j if j < 4 else j + 3             # batch index (7, 8 for the last two)
            r_out, r_m, r_n = ref[i % 3]
            assert n == r_n, i
            for f in range(F):
                assert np.array_equal(out[f][0], r_out[f][0]) and np.array_equal(out[f][1], r_out[f][1]), (i, f)
                if f:
                    assert np.array_equal(m[f], r_m[f]), (i, f)
    finally:
        hs.close()
        for b in bufs:
            b.free()


# ------------------------------------------------------------------ local-map projection search
def localmap_both(ctx, oracle_mod, ex, cur_k, cur_d, cur_ur, cur_obs, mp, th=3.0, nnratio=0.8):
    """coeb_match_localmap vs oracle.search_local_map (ORBmatcher.cc:44-129), bit-exact."""
    import coeb_front
    cam_o = oracle_mod.camera(ex, 640, 480, synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
    obs = np.full(len(cur_k), -1, np.int32) if cur_obs is None else cur_obs
    nm_ref, m_ref = oracle_mod.search_local_map(cam_o, cur_k, cur_d, cur_ur, obs, mp, th, nnratio)
    cam = coeb_front.make_camera(synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF, 640, 480)
    F = coeb_front.Frame(cur_k, cur_d, cur_ur)
    if cur_obs is not None:
        F.mvpMapPointObs = cur_obs.copy()
    lm = coeb_front.LocalMap(mp["in_view"], mp["proj_x"], mp["proj_y"], mp["proj_xr"], mp["level"], mp["view_cos"],
                             mp["descriptor"], mp["observations"])
    nm = coeb_front.ORBmatcher(nnratio, ctx=ctx).SearchByProjection(F, lm, th, camera=cam)
    got = F.mvpMapPoints
    assert nm == nm_ref, (nm, nm_ref)
    assert np.array_equal(got, m_ref), int(np.sum(got != m_ref))
    return nm


def localmap_path(ctx):
    """(path, iterations) of the last coeb_match_localmap: 0 parallel claims, 1 forced
    sequential, 2 candidate-list overflow, 3 no convergence."""
    p = ctx.debug_read("localmap_path").view(np.int32)
    return int(p[0]), int(p[1])


@pytest.fixture(scope="module")
def local_scene(oracle_mod, ex, pair):
    r1, ur1, last = pair
    Tc = synth.motion_pose()
    return r1, ur1, last, Tc


@pytest.mark.parametrize("seed,th,nnratio", [(0, 3.0, 0.8), (1, 1.0, 0.8), (2, 5.0, 0.8), (3, 3.0, 1.0),
                                             (4, 3.0, 0.6)])
def test_localmap_matches_oracle(ctx, oracle_mod, ex, local_scene, seed, th, nnratio):
    r1, ur1, last, Tc = local_scene
    mp = synth.make_local_map(last["xw"], last["mp_desc"], last["keys_un"]["octave"], Tc, 640, 480, seed=seed)
    rng = np.random.default_rng(100 + seed)
    nm = localmap_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], ur1, None, mp, th, nnratio)
    assert nm > 50
    assert localmap_path(ctx)[0] == 0          # the parallel claim resolution produced this
    # keypoints already holding MapPoints (Observations() -1 / 0 / >0, ORBmatcher.cc:86-88)
    obs = rng.choice(np.array([-1, -1, 0, 2], np.int32), len(r1["kps"])).astype(np.int32)
    localmap_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], ur1, obs, mp, th, nnratio)
    # monocular current frame (mvuRight < 0 everywhere)
    localmap_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], np.full(len(ur1), -1, np.float32), obs, mp, th, nnratio)


def test_localmap_paths_agree(ctx, oracle_mod, ex, local_scene, monkeypatch):
    """Parallel claim fixpoint and the literal sequential loop (COEB_MATCH_SEQUENTIAL) agree."""
    r1, ur1, last, Tc = local_scene
    mp = synth.make_local_map(last["xw"], last["mp_desc"], last["keys_un"]["octave"], Tc, 640, 480, seed=9,
                              dup_frac=0.8)
    obs = np.random.default_rng(9).choice(np.array([-1, 0, 3], np.int32), len(r1["kps"])).astype(np.int32)
    for seq in (False, True):
        if seq:
            monkeypatch.setenv("COEB_MATCH_SEQUENTIAL", "1")
        localmap_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], ur1, obs, mp, 3.0, 0.8)
        assert localmap_path(ctx)[0] == (1 if seq else 0)
        localmap_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], ur1, None, mp, 5.0, 0.9)
        assert localmap_path(ctx)[0] == (1 if seq else 0)
    monkeypatch.delenv("COEB_MATCH_SEQUENTIAL")


def test_localmap_edge_cases(ctx, oracle_mod, ex, local_scene):
    import coeb_front
    r1, ur1, last, Tc = local_scene
    mp = synth.make_local_map(last["xw"], last["mp_desc"], last["keys_un"]["octave"], Tc, 640, 480, seed=5)
    empty = {k: v[:0] for k, v in mp.items()}
    assert localmap_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], ur1, None, empty) == 0
    k0 = r1["kps"][:0]
    assert localmap_both(ctx, oracle_mod, ex, k0, r1["desc"][:0], ur1[:0], None, mp) == 0
    off = dict(mp)
    off["in_view"] = np.zeros_like(mp["in_view"])
    assert localmap_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], ur1, None, off) == 0
    # every point predicted at level 0 (window levels [-1, 0]) or at the top level
    for lv in (0, 7):
        v = dict(mp)
        v["level"] = np.where(mp["in_view"] > 0, lv, -1).astype(np.int32)
        localmap_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], ur1, None, v, 5.0)
    # a level outside the pyramid on a point in view is rejected, not read out of bounds
    bad = dict(mp)
    bad["level"] = mp["level"].copy()
    bad["level"][np.argmax(mp["in_view"])] = 8
    with pytest.raises(coeb_front.CoebError):
        localmap_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], ur1, None, bad)


def test_localmap_crowded_windows(ctx, oracle_mod, ex):
    """Repetitive texture + a wide window: candidate lists overflow (sequential fallback)."""
    yy, xx = np.indices((480, 640))
    base = (((yy // 12) + (xx // 12)) % 2 * 200 + 30).astype(np.int16)
    rng = np.random.default_rng(8)
    f0 = np.clip(base + rng.integers(-6, 7, base.shape), 0, 255).astype(np.uint8)
    f1 = np.clip(np.roll(base, (1, 2), axis=(0, 1)) + rng.integers(-6, 7, base.shape), 0, 255).astype(np.uint8)
    r0, r1 = ex.extract(f0), ex.extract(f1)
    depth = synth.make_depth(640, 480)
    last = oracle_mod.mapframe_from_extraction(r0["kps"], r0["desc"], depth, synth.TUM_FX, synth.TUM_FY,
                                               synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
    ur1, _ = oracle_mod.stereo_from_rgbd(r1["kps"], depth, synth.TUM_BF)
    mp = synth.make_local_map(last["xw"], last["mp_desc"], last["keys_un"]["octave"], synth.motion_pose(), 640, 480,
                              seed=3)
    paths = []
    for th in (3.0, 12.0):
        localmap_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], ur1, None, mp, th)
        paths.append(localmap_path(ctx)[0])
    assert paths == [0, 2], paths


# ------------------------------------------------------------------ relocalisation projection search
def keyframe_both(ctx, oracle_mod, ex, cur_k, cur_d, cur_has, kf, Tcw, th=10.0, orb_dist=100, check_ori=True,
                  already=()):
    """coeb_match_keyframe vs oracle.search_keyframe (ORBmatcher.cc:1473-1600), bit-exact."""
    import coeb_front
    cam_o = oracle_mod.camera(ex, 640, 480, synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
    kv = dict(kf)
    kv["valid"] = kf["valid"].copy()
    for i in already:
        kv["valid"][i] = 0
    has = np.zeros(len(cur_k), np.uint8) if cur_has is None else cur_has
    nm_ref, m_ref = oracle_mod.search_keyframe(cam_o, cur_k, cur_d, has, kv, Tcw, th, orb_dist, check_ori)
    cam = coeb_front.make_camera(synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF, 640, 480)
    F = coeb_front.Frame(cur_k, cur_d, Tcw=Tcw)
    if cur_has is not None:
        F.mvpMapPoints = np.where(cur_has > 0, 10 ** 6, -1).astype(np.int32)    # a MapPoint from elsewhere
    kp = coeb_front.KeyFramePoints(kf["valid"], kf["world_pos"], kf["descriptor"], kf["max_distance"],
                                   kf["min_distance"], kf["angle"])
    nm = coeb_front.ORBmatcher(0.75, check_ori, ctx=ctx).SearchByProjection(F, kp, set(already), th, orb_dist, cam)
    got = np.where(F.mvpMapPoints == 10 ** 6, -1, F.mvpMapPoints)
    assert nm == nm_ref, (nm, nm_ref)
    assert np.array_equal(got, m_ref), int(np.sum(got != m_ref))
    return nm


def search_path(ctx):
    p = ctx.debug_read("search_path").view(np.int32)
    return int(p[0]), int(p[1])


@pytest.mark.parametrize("seed,th,orb_dist", [(0, 10.0, 100), (1, 3.0, 64), (2, 10.0, 50), (3, 25.0, 100)])
def test_keyframe_matches_oracle(ctx, oracle_mod, ex, pair, seed, th, orb_dist):
    r1, ur1, last = pair
    kf = synth.make_keyframe_points(last["xw"], last["mp_desc"], last["keys_un"]["octave"], last["keys_un"]["angle"],
                                    seed=seed)
    kf["valid"] &= last_has(last, kf)
    rng = np.random.default_rng(200 + seed)
    for T in (synth.motion_pose(), synth.rotated_pose(1.5, axis=seed % 3)):
        nm = keyframe_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], None, kf, T, th, orb_dist)
        assert search_path(ctx)[0] == 0
        has = (rng.random(len(r1["kps"])) < 0.3).astype(np.uint8)
        keyframe_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], has, kf, T, th, orb_dist,
                      already=rng.choice(len(kf["valid"]), 50, replace=False))
        keyframe_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], None, kf, T, th, orb_dist, check_ori=False)
    assert nm > 20


def last_has(last, kf):
    """Valid only where the LastFrame keypoint had a MapPoint (depth > 0); distractors stay."""
    v = np.ones(len(kf["valid"]), np.uint8)
    v[:len(last["has_mp"])] = last["has_mp"]
    return v


def test_keyframe_paths_and_edges(ctx, oracle_mod, ex, pair, monkeypatch):
    import coeb_front
    r1, ur1, last = pair
    kf = synth.make_keyframe_points(last["xw"], last["mp_desc"], last["keys_un"]["octave"], last["keys_un"]["angle"],
                                    seed=7)
    kf["valid"] &= last_has(last, kf)
    T = synth.motion_pose()
    monkeypatch.setenv("COEB_MATCH_SEQUENTIAL", "1")
    keyframe_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], None, kf, T)
    assert search_path(ctx)[0] == 1
    monkeypatch.delenv("COEB_MATCH_SEQUENTIAL")
    # wide window on repetitive descriptors: list overflow -> literal loop
    dup = dict(kf)
    dup["descriptor"] = np.repeat(kf["descriptor"][:1], len(kf["valid"]), axis=0)
    keyframe_both(ctx, oracle_mod, ex, r1["kps"], np.repeat(kf["descriptor"][:1], len(r1["kps"]), axis=0), None,
                  dup, T, th=200.0)
    assert search_path(ctx)[0] == 2
    # empty keyframe / empty frame / every point behind or outside
    empty = {k: v[:0] for k, v in kf.items()}
    assert keyframe_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], None, empty, T) == 0
    assert keyframe_both(ctx, oracle_mod, ex, r1["kps"][:0], r1["desc"][:0], None, kf, T) == 0
    away = synth.rotated_pose(180.0, axis=1, t=(0, 0, 0))
    keyframe_both(ctx, oracle_mod, ex, r1["kps"], r1["desc"], None, kf, away)
    with pytest.raises(ValueError):
        coeb_front.KeyFramePoints(kf["valid"], kf["world_pos"], kf["descriptor"], kf["max_distance"],
                                  kf["min_distance"], kf["angle"][:-1])


# ------------------------------------------------------------------ Optimizer::PoseOptimization
def pose_both(ctx, oracle_mod, P, cam=None):
    """coeb_pose_optimization vs oracle.pose_optimization: pose bits, outlier flags and the
    inlier count identical (same canonical operations and reduction order)."""
    import coeb_front
    isg = np.array(ctx.tables().inv_sigma2[:8], np.float32)
    intr = P.get("cam", (synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF))
    nin_ref, T_ref, out_ref = oracle_mod.pose_optimization(P["kps"], P["has_mp"], P["xw"], P["ur"], isg, *intr,
                                                           P["Tcw_init"])
    cam = cam or coeb_front.make_camera(*intr, 640, 480)
    F = coeb_front.Frame(P["kps"], np.zeros((len(P["kps"]), 32), np.uint8), P["ur"], Tcw=P["Tcw_init"])
    F.mvpMapPoints = np.where(P["has_mp"] > 0, 0, -1).astype(np.int32)
    F.mvMapPointPos = P["xw"]
    nin = coeb_front.Optimizer.PoseOptimization(F, cam, ctx)
    assert nin == nin_ref, (nin, nin_ref)
    assert np.array_equal(F.mTcw.view(np.uint32), T_ref.view(np.uint32)), (F.mTcw, T_ref)
    has = P["has_mp"] > 0
    assert np.array_equal(F.mvbOutlier[has], out_ref[has])
    return nin


@pytest.mark.parametrize("seed,kw", [(0, {}), (1, {"outlier_frac": 0.4}), (2, {"mono_frac": 1.0}),
                                     (3, {"mono_frac": 0.0, "n": 1500}), (4, {"noise": 3.0}),
                                     (5, {"init_err": (0.15, 0.3)})])
def test_pose_optimization_matches_oracle(ctx, oracle_mod, seed, kw):
    P = synth.make_pose_problem(seed=seed, **kw)
    assert pose_both(ctx, oracle_mod, P) > 0


def test_pose_optimization_edges(ctx, oracle_mod):
    P = synth.make_pose_problem(n=40, seed=9)
    for k in (0, 2, 5, 9, 12):                       # < 3 (untouched), < 10 (one round), >= 10
        Q = dict(P)
        Q["has_mp"] = np.zeros_like(P["has_mp"])
        Q["has_mp"][:k] = 1
        pose_both(ctx, oracle_mod, Q)


def test_pose_optimization_rho_zero(ctx, oracle_mod):
    """Zero residuals at the entry pose: g2o's scale += 1e-3 gives rho == 0 and Terminate
    (test_oracle_kat.py::test_pose_optimization_rho_zero_terminates); the kernel agrees, and so
    it does from a perturbed start."""
    from test_oracle_kat import exact_pose_problem
    P = exact_pose_problem()
    assert pose_both(ctx, oracle_mod, P) == len(P["kps"])
    Q = dict(P)
    Q["Tcw_init"] = np.eye(4, dtype=np.float32)
    Q["Tcw_init"][0, 3] = 0.01
    assert pose_both(ctx, oracle_mod, Q) == len(P["kps"])


# ------------------------------------------------------------------ Frame ingest helpers
def test_undistort_keypoints(ctx, oracle_mod, ex, pair):
    import coeb_front
    r1, _, _ = pair
    k = r1["kps"]
    cam = coeb_front.make_camera(517.306408, 516.469215, 318.643040, 255.313989, synth.TUM_BF, 640, 480)
    for dist in ((0.262383, -0.953104, -0.005358, 0.002628, 1.163314), (0.2312, -0.7849, -0.0033, -0.0001, 0.0),
                 (0.0, 0.5, 0.1, 0.1, 0.1)):
        got = coeb_front.UndistortKeyPoints(ctx, k, cam, dist)
        ref = oracle_mod.undistort_keypoints(k, 517.306408, 516.469215, 318.643040, 255.313989, dist)
        assert got.tobytes() == ref.tobytes(), dist
    assert len(coeb_front.UndistortKeyPoints(ctx, k[:0], cam, (0.1, 0, 0, 0, 0))) == 0



def _chain_oracle(oracle_mod, ex, frames, boxes, Tpred, stride, isg, nkf=2):
    """The configs[4] loop frame by frame on the oracle: Frame ctor (T_M from the previous frame,
    blur flags, masked extraction) when boxes is given, else the plain extraction; then
    track_frame (motion model + TrackLocalMap)."""
    F, H, W = frames.shape
    depth = synth.make_depth(W, H)
    cam_o = oracle_mod.camera(ex, W, H, synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
    ext, res = [], [None]
    for f in range(F):
        if boxes is None:
            ext.append(ex.extract(frames[f]))
            continue
        if f == 0:
            tm, bl = np.zeros((0, 2), np.float32), np.zeros(len(boxes[0]), np.int32)
        else:
            tm = oracle_mod.process_moving_object(frames[f - 1], frames[f])
            tm = np.zeros((0, 2), np.float32) if tm is None else tm
            bl, _ = oracle_mod.blur_flags(frames[f], boxes[f])
        ext.append(ex.extract(frames[f], boxes[f], tm, bl))
    mfs = [oracle_mod.mapframe_from_extraction(e["kps"], e["desc"], depth, synth.TUM_FX, synth.TUM_FY, synth.TUM_CX,
                                               synth.TUM_CY, synth.TUM_BF) for e in ext]
    for f in range(1, F):
        ur, _ = oracle_mod.stereo_from_rgbd(ext[f]["kps"], depth, synth.TUM_BF)
        prev2 = mfs[f - 2] if (nkf >= 2 and f >= 2) else None
        T_last = res[f - 1]["T1"] if f >= 2 else np.eye(4, dtype=np.float32)
        res.append(oracle_mod.track_frame(cam_o, isg, ext[f], ur, mfs[f - 1], prev2, Tpred[f], T_last, stride,
                                          fx=synth.TUM_FX, fy=synth.TUM_FY, cx=synth.TUM_CX, cy=synth.TUM_CY,
                                          bf=synth.TUM_BF))
    return ext, res


def _check_chain(bp, ext, res, F):
    out, matches, nms = bp.results()
    T1, nin1, _ = bp.pose_results()
    tr = bp.track_results()
    states = []
    for f in range(1, F):
        r = res[f]
        assert np.array_equal(out[f][1], ext[f]["desc"]), f
        assert nms[f] == r["nmatches"] and np.array_equal(matches[f], r["match"]), f
        assert np.array_equal(T1[f].view(np.uint32), r["T1"].view(np.uint32)), f
        assert nin1[f] == r["nin1"], f
        assert tr["state"][f] == r["state"], (f, tr["state"][f], r["state"])
        states.append(r["state"])
        if r["nmatches"] >= 20:
            assert tr["nmatches_map"][f] == r["nmatches_map"], f
        if r["state"] == 0:
            assert tr["ninliers"][f] == 0 and np.array_equal(tr["T"][f].view(np.uint32), r["T1"].view(np.uint32)), f
            continue
        assert tr["nlocal"][f] == r["nlocal"], (f, tr["nlocal"][f], r["nlocal"])
        assert np.array_equal(tr["local_match"][f], r["local_match"]), f
        assert tr["ninliers"][f] == r["ninliers"], (f, tr["ninliers"][f], r["ninliers"])
        assert np.array_equal(tr["T"][f].view(np.uint32), r["T"].view(np.uint32)), f
        h2 = r["has2"] > 0
        assert np.array_equal(tr["outlier"][f][h2], r["outlier"][h2]), f
    return states, tr


def test_batch_track_local_map_matches_oracle(oracle_mod, ex):
    """BASELINE configs[4] as the loop: TrackWithMotionModel (match + retry + PoseOptimization +
    outlier discard) then TrackLocalMap (local map of KeyFrames f-1, f-2 through isInFrustum,
    SearchByProjection th 3, second PoseOptimization) for every frame of the device batch,
    against the oracle frame by frame (Tracking.cc:933-1047, 1222-1272).  Frame 3's prediction
    is 180 degrees off: the motion model fails there, and frame 4's local map still uses frame
    3's (unoptimised) pose for KeyFrame 2."""
    from coeb_front.pipeline import BatchPipeline
    F = 7
    fr = synth.make_frames(640, 480, F, seed=4242)
    Tcw = np.stack([synth.motion_pose()] * F)
    Tcw[3] = synth.rotated_pose(180.0, axis=1, t=(0, 0, 0))
    bp = BatchPipeline(640, 480, F)
    try:
        bp.load(fr, Tcw=Tcw)
        bp.run(track=True)
        bp.synchronize()
        stride = bp.ctx.batch_results()[3]
        isg = np.array(bp.ctx.tables().inv_sigma2[:8], np.float32)
        ext, res = _chain_oracle(oracle_mod, ex, fr, None, Tcw, stride, isg)
        states, tr = _check_chain(bp, ext, res, F)
        assert states.count(2) >= F - 3 and states[2] == 0                  # frame 3 lost
        assert sum(tr["nlocal"][f] for f in range(1, F) if states[f - 1] == 2) > 0
        # pipelined: three back-to-back steps leave the single-step results
        for _ in range(3):
            bp.run(track=True)
        tr2 = bp.track_results()
        assert tr2["ninliers"] == tr["ninliers"] and tr2["nlocal"] == tr["nlocal"]
        assert np.array_equal(tr2["T"][1:].view(np.uint32), tr["T"][1:].view(np.uint32))
    finally:
        bp.close()


def test_batch_grab_rgbd_loop_matches_oracle(oracle_mod, ex):
    """The whole configs[4] loop on a moving-object sequence: Frame ctor on the device (T_M from
    ProcessMovingObject of the previous frame, blur flags, masked extraction), then the motion
    model and TrackLocalMap, each frame against the oracle.  The nearer panels move 2-3x the
    camera prediction, so the optimisations see real outliers.  nkf = 1 (local map = KeyFrame
    f-1 only) is checked on the same batch."""
    from coeb_front.pipeline import BatchPipeline
    F = 6
    frames, obj = synth.moving_object_sequence(640, 480, F, seed=8)
    boxes = [obj[f][None, :] for f in range(F)]
    Tcw = np.stack([synth.motion_pose()] * F)
    bp = BatchPipeline(640, 480, F)
    try:
        bp.load(frames, Tcw=Tcw)
        bp.set_frame_boxes(boxes)
        for nkf in (2, 1):
            bp.run(frame=True, track=True, nkf=nkf)
            bp.synchronize()
            stride = bp.ctx.batch_results()[3]
            isg = np.array(bp.ctx.tables().inv_sigma2[:8], np.float32)
            ext, res = _chain_oracle(oracle_mod, ex, frames, boxes, Tcw, stride, isg, nkf=nkf)
            states, tr = _check_chain(bp, ext, res, F)
            assert states.count(2) >= F - 2, states
            assert any(r["nlocal"] > 0 for r in res[1:])
            assert any(((r["outlier"] > 0) & (r["has2"] > 0)).any() for r in res[1:] if r["state"] > 0)
    finally:
        bp.close()


@pytest.mark.parametrize("ch,order,dt,W,H", [(3, 1, np.uint16, 320, 240), (3, 0, np.uint16, 320, 240),
                                              (4, 1, np.float32, 320, 240), (1, 1, np.float32, 320, 240),
                                              (4, 0, np.uint16, 320, 240), (3, 1, np.uint16, 324, 242),
                                              (1, 1, np.float32, 324, 242)])
def test_rgbd_preprocess_batch_matches_oracle(oracle_mod, ch, order, dt, W, H):
    """GrabImageRGBD's conversions over a device batch (coeb_rgbd_preprocess_batch_device) vs
    the oracle frame by frame: RGB/BGR/RGBA/BGRA/gray images, 16U depth with 1/5000 and 32F
    depth with factor 1 (passthrough, Tracking.cc:227) or 1/5000.  320x240 frames take the
    16-pixels-per-thread kernel; 324x242 (W*H not a multiple of 16) the 4-pixel one."""
    import coeb_front as cf
    from coeb_front.pipeline import BatchPipeline
    F = 3
    rng = np.random.default_rng(ch * 10 + order)
    img = rng.integers(0, 256, (F, H, W, ch) if ch > 1 else (F, H, W), dtype=np.uint8)
    if dt == np.uint16:
        dep, fac = rng.integers(0, 65536, (F, H, W), dtype=np.uint16), 1.0 / 5000.0
    else:
        dep = rng.uniform(0, 8, (F, H, W)).astype(np.float32)
        fac = 1.0 if ch == 1 else 1.0 / 5000.0
    bp = BatchPipeline(W, H, F)
    try:
        bp.load_rgbd(img, dep, fac, rgb_order=order)
        bp.run(rgbd=True, match=False)
        bp.synchronize()
        gray = bp.ctx.download(bp.gray.ptr, F * H * W, np.uint8).reshape(F, H, W)
        depth = bp.ctx.download(bp.depth.ptr, 4 * F * H * W, np.float32).reshape(F, H, W)
        for f in range(F):
            assert np.array_equal(gray[f], oracle_mod.image_to_gray(img[f], order)), f
            assert np.array_equal(depth[f].view(np.uint32), oracle_mod.depth_to_float(dep[f], np.float32(fac)).view(np.uint32)), f
        # bad arguments fail loudly
        with pytest.raises(RuntimeError):
            bp.ctx.rgbd_preprocess_batch_device(bp.raw[0].ptr, 2, 1, 0, 0, 1.0, F, W, H, bp.gray.ptr, 0)
        with pytest.raises(RuntimeError):
            bp.ctx.rgbd_preprocess_batch_device(bp.raw[0].ptr, ch, 1, 0, 0, 1.0, F, W - 2, H, bp.gray.ptr, 0)
        assert cf.DEPTH_F32 == 1
    finally:
        bp.close()


def test_batch_grab_rgbd_loop_sharded_equals_unsharded():
    """bench --config D shards the sequence with a 3-frame halo (dist.shard_frames(halo=3)):
    the counted frames of a shard must come out bit-identical to the same frames of the
    unsharded batch through the whole loop (RGB-D conversion, Frame ctor, motion model,
    TrackLocalMap)."""
    from coeb_front.dist import shard_frames
    from coeb_front.pipeline import BatchPipeline
    import bench
    G = 8
    full = None
    for world, rank in ((1, 0), (2, 1)):
        first, F, nm = shard_frames(G, world, rank, halo=3)
        bp = BatchPipeline(640, 480, F)
        try:
            bench.load_batch(bp, bench.CONFIGS["D"], 640, 480, F, first)
            bp.run(**bench.step_kwargs(bench.CONFIGS["D"]))
            bp.synchronize()
            out, _, nms = bp.results()
            tr = bp.track_results()
            res = {first + f: (out[f][0], out[f][1], nms[f], tr["T"][f].copy(), tr["ninliers"][f], tr["nlocal"][f],
                               tr["local_match"][f], tr["state"][f]) for f in range(F - nm, F)}
        finally:
            bp.close()
        if full is None:
            full = res
            assert sorted(res) == list(range(1, G + 1))
            assert sum(1 for v in res.values() if v[7] == 2) >= G - 1
            continue
        assert first == 2 and sorted(res) == list(range(5, G + 1))
        for g, v in res.items():
            w = full[g]
            assert np.array_equal(v[0], w[0]) and np.array_equal(v[1], w[1]) and v[2] == w[2], g
            assert np.array_equal(v[3].view(np.uint32), w[3].view(np.uint32)), g
            assert v[4:6] == w[4:6] and np.array_equal(v[6], w[6]) and v[7] == w[7], g


def test_extract_null_arrays(ctx, oracle_mod, ex):
    """coeb_extract's array arguments: a null blur_flag with nblur > 0 reads as all-zero flags
    (the reference's missing flags), null boxes / T_M with a nonzero count fail loudly."""
    import ctypes as C
    import coeb_front as cf
    img = synth.make_frames(640, 480, 1, seed=31)[0]
    boxes, tm, _ = synth.dynamic_inputs(640, 480, seed=3)
    cap = ctx.max_keypoints(640, 480)
    kps = np.zeros(cap, cf.KEYPOINT_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    n = C.c_int()
    L = cf.lib()
    rc = L.coeb_extract(ctx.h, img.ctypes.data, 640, 480, 640, boxes.ctypes.data, len(boxes), tm.ctypes.data, len(tm),
                        None, 2, kps.ctypes.data, desc.ctypes.data, cap, C.byref(n))
    assert rc == 0
    r = ex.extract(img, boxes, tm, np.zeros(len(boxes), np.int32))
    assert n.value == len(r["kps"]) and np.array_equal(desc[:n.value], r["desc"])
    for bad in ((None, len(boxes), tm.ctypes.data, len(tm)), (boxes.ctypes.data, len(boxes), None, len(tm))):
        rc = L.coeb_extract(ctx.h, img.ctypes.data, 640, 480, 640, bad[0], bad[1], bad[2], bad[3], None, 0,
                            kps.ctypes.data, desc.ctypes.data, cap, C.byref(n))
        assert rc == cf.COEB_EINVAL if hasattr(cf, "COEB_EINVAL") else rc != 0
