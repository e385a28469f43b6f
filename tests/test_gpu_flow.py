"""Frame::ProcessMovingObject (src/Frame.cc:311-393) on the HIP path vs the CPU oracle, stage by
stage and end to end (MI355X only).  Every comparison is bit-exact: corner and flow coordinates
are float32 and F is float64, produced by the same canonical arithmetic;
OpenCV itself is absent, so parity against it is unpinned."""
import numpy as np
import pytest

import coeb_front as cf
from coeb_front import synth

pytestmark = pytest.mark.gpu


def pairs():
    out = []
    for seed in range(3):
        prev, cur, _ = synth.moving_object_pair(640, 480, seed)
        out.append(("obj%d" % seed, prev, cur))
    fr = synth.make_frames(640, 480, 2, seed=1003)
    out.append(("tum", fr[0], fr[1]))
    return out


PAIRS = pairs()


def eq(a, b, tag):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape, (tag, a.shape, b.shape)
    bad = np.nonzero((a != b).reshape(len(a), -1).any(axis=1))[0] if len(a) else []
    assert len(bad) == 0, (tag, len(bad), a[bad[:3]], b[bad[:3]])


@pytest.mark.parametrize("tag,prev,cur", PAIRS, ids=[p[0] for p in PAIRS])
def test_good_features(ctx, oracle_mod, tag, prev, cur):
    got = cf.GoodFeaturesToTrack(ctx, prev)
    ref = oracle_mod.good_features(prev)
    assert len(ref) > 50
    eq(got, ref, tag)


def test_good_features_edges(ctx, oracle_mod):
    flat = np.full((96, 128), 77, np.uint8)
    assert len(cf.GoodFeaturesToTrack(ctx, flat)) == 0
    assert len(oracle_mod.good_features(flat)) == 0
    small = synth.moving_object_pair(640, 480, 5)[0][100:164, 200:296].copy()
    eq(cf.GoodFeaturesToTrack(ctx, small), oracle_mod.good_features(small), "small")
    for mc in (1, 17, 250):                            # maxCorners cut of the greedy order
        eq(cf.GoodFeaturesToTrack(ctx, PAIRS[0][1], max_corners=mc), oracle_mod.good_features(PAIRS[0][1], mc), mc)
    # equal responses: a regular grid of identical corners exercises the index tie-break
    grid = np.zeros((120, 160), np.uint8)
    for y in range(10, 110, 20):
        for x in range(10, 150, 20):
            grid[y:y + 10, x:x + 10] = 200
    eq(cf.GoodFeaturesToTrack(ctx, grid), oracle_mod.good_features(grid), "grid")


@pytest.mark.parametrize("tag,prev,cur", PAIRS, ids=[p[0] for p in PAIRS])
def test_corner_subpix(ctx, oracle_mod, tag, prev, cur):
    pts = oracle_mod.good_features(prev)
    eq(cf.CornerSubPix(ctx, prev, pts), oracle_mod.corner_subpix(prev, pts), tag)


def test_corner_subpix_border(ctx, oracle_mod):
    prev = PAIRS[0][1]
    h, w = prev.shape
    pts = np.array([[1, 1], [w - 2, h - 2], [0.5, 3.25], [w - 1.5, 40.75], [11.2, 11.9], [320.4, 2.0],
                    [630.1, 470.2], [5, h - 1]], np.float32)
    eq(cf.CornerSubPix(ctx, prev, pts), oracle_mod.corner_subpix(prev, pts), "border")


@pytest.mark.parametrize("tag,prev,cur", PAIRS, ids=[p[0] for p in PAIRS])
def test_lk(ctx, oracle_mod, tag, prev, cur):
    pts = oracle_mod.corner_subpix(prev, oracle_mod.good_features(prev))
    nx, st = cf.CalcOpticalFlowPyrLK(ctx, prev, cur, pts)
    rnx, rst = oracle_mod.lk_pyr(prev, cur, pts)
    eq(st, rst, tag + " status")
    eq(nx, rnx, tag + " next")


def test_lk_edges(ctx, oracle_mod):
    prev, cur = PAIRS[1][1], PAIRS[1][2]
    h, w = prev.shape
    # (x.5001, y.5001): at level 0 the window origin sits 1e-4 past a pixel, so the rounded weights
    # give iw11 = 16384 - 16381 - 2 - 2 = -1 (the taps are signed)
    pts = np.array([[0, 0], [w - 1, h - 1], [-3, 10], [w + 40, 20], [2.5, h - 1.5], [320, 240], [11, 470],
                    [100.5001, 200.5001], [320.5001, 240.5001]], np.float32)
    nx, st = cf.CalcOpticalFlowPyrLK(ctx, prev, cur, pts)
    rnx, rst = oracle_mod.lk_pyr(prev, cur, pts)
    eq(st, rst, "status")
    eq(nx[rst == 1], rnx[rst == 1], "next")
    # a flat pair: every point fails the minimum-eigenvalue test
    flat = np.full((120, 160), 90, np.uint8)
    _, st = cf.CalcOpticalFlowPyrLK(ctx, flat, flat, np.array([[80, 60], [20, 30]], np.float32))
    assert not st.any()


@pytest.mark.parametrize("tag,prev,cur", PAIRS, ids=[p[0] for p in PAIRS])
def test_moving_tail(ctx, oracle_mod, tag, prev, cur):
    pts = oracle_mod.corner_subpix(prev, oracle_mod.good_features(prev))
    nx, st = oracle_mod.lk_pyr(prev, cur, pts)
    tm, st2, F, nf = cf.MovingTail(ctx, prev, cur, pts, nx, st)
    rtm, rst2, rF, rnf = oracle_mod.moving_tail(prev, cur, pts, nx, st)
    eq(st2, rst2, tag + " state")
    assert nf == rnf
    assert (F is None) == (rF is None)
    if F is not None:
        assert np.array_equal(F, rF), (F, rF)
        eq(tm, rtm, tag + " T_M")


@pytest.mark.parametrize("npts", [0, 5, 7, 9, 12, 14, 15, 40])
def test_moving_tail_small_sets(ctx, oracle_mod, npts):
    """n < 7 (empty F), n == 7 (run7Point), 8..14 (LMeDS), >= 15 (RANSAC)"""
    prev, cur = PAIRS[2][1], PAIRS[2][2]
    pts = oracle_mod.corner_subpix(prev, oracle_mod.good_features(prev))
    nx, st = oracle_mod.lk_pyr(prev, cur, pts)
    keep = np.nonzero(st)[0][:npts]
    p, q, s = pts[keep], nx[keep], st[keep]
    tm, st2, F, nf = cf.MovingTail(ctx, prev, cur, p, q, s)
    rtm, rst2, rF, rnf = oracle_mod.moving_tail(prev, cur, p, q, s)
    assert nf == rnf
    eq(st2, rst2, "state")
    assert (F is None) == (rF is None)
    if npts < 7:
        assert F is None
    if F is not None:
        assert np.array_equal(F, rF)
        eq(tm, rtm, "T_M")


@pytest.mark.parametrize("threads", [256, 512, 1024])
def test_moving_tail_fm_thread_counts(ctx, oracle_mod, monkeypatch, threads):
    """k_fm with 256 / 512 / 1024 threads per pair (COEB_FM_THREADS; the default is 128): every
    pair's SAD states, F and T_M against the oracle, and the LMeDS (9, 12 points) and RANSAC (15,
    40) branches on the small sets."""
    monkeypatch.setenv("COEB_FM_THREADS", str(threads))
    for tag, prev, cur in PAIRS:
        pts = oracle_mod.corner_subpix(prev, oracle_mod.good_features(prev))
        nx, st = oracle_mod.lk_pyr(prev, cur, pts)
        cases = [(pts, nx, st)]
        if tag == PAIRS[2][0]:
            for npts in (9, 12, 15, 40):
                keep = np.nonzero(st)[0][:npts]
                cases.append((pts[keep], nx[keep], st[keep]))
        for p, q, s_ in cases:
            tm, st2, F, nf = cf.MovingTail(ctx, prev, cur, p, q, s_)
            rtm, rst2, rF, rnf = oracle_mod.moving_tail(prev, cur, p, q, s_)
            eq(st2, rst2, tag + " state")
            assert nf == rnf
            assert (F is None) == (rF is None)
            if F is not None:
                assert np.array_equal(F, rF), (tag, len(p))
                eq(tm, rtm, tag + " T_M")


@pytest.mark.parametrize("tag,prev,cur", PAIRS, ids=[p[0] for p in PAIRS])
def test_process_moving_object(ctx, oracle_mod, tag, prev, cur):
    tm, d = cf.ProcessMovingObject(ctx, prev, cur, debug=True)
    ref = oracle_mod.process_moving_object(prev, cur)
    assert (tm is None) == (ref is None)
    if ref is not None:
        eq(tm, ref, tag)
    pts = oracle_mod.good_features(prev)
    eq(d["corners_raw"], pts, "gf")
    sp = oracle_mod.corner_subpix(prev, pts)
    eq(d["corners"], sp, "subpix")
    rnx, rst = oracle_mod.lk_pyr(prev, cur, sp)
    eq(d["status"], rst, "lk status")


def test_process_moving_object_flags_object(ctx):
    """size-independent property: T_M of the layered scene lies on the moving object"""
    for seed in range(3):
        prev, cur, (x0, y0, x1, y1) = synth.moving_object_pair(640, 480, seed)
        tm = cf.ProcessMovingObject(ctx, prev, cur)
        assert tm is not None and len(tm) >= 20
        inb = (tm[:, 0] >= x0 - 2) & (tm[:, 0] < x1 + 2) & (tm[:, 1] >= y0 - 2) & (tm[:, 1] < y1 + 2)
        assert inb.mean() > 0.8, (seed, inb.mean())


def test_frame_batch_matches_oracle_frame_by_frame(oracle_mod):
    """The RGB-D Frame constructor on a device batch (coeb_frame_batch_device, Frame.cc:157-214):
    for every frame f, ProcessMovingObject(frame f-1, frame f) -> T_M, the boxes' blur flags
    (frame 0: the sequence's first frame, no T_M and flags 0) and the masked extraction, against
    the oracle run frame by frame; then the batch matcher follows on those keypoints."""
    from coeb_front.pipeline import BatchPipeline
    F = 6
    frames, obj = synth.moving_object_sequence(640, 480, F, seed=3)
    boxes = [np.stack([obj[f], np.float32([420, 60, 600, 200])]) for f in range(F)]   # object + a static panel
    bp = BatchPipeline(640, 480, F)
    try:
        bp.load(frames, Tcw=np.stack([synth.motion_pose()] * F))
        bp.set_frame_boxes(boxes)
        bp.run(frame=True)
        bp.synchronize()
        out, matches, nms = bp.results()
        tms, flags = bp.ctx.batch_frame_results(F, 2 * F)
        ex = oracle_mod.Extractor()
        ntm_total = 0
        for f in range(F):
            if f == 0:
                tm_ref, blur_ref = np.zeros((0, 2), np.float32), np.zeros(2, np.int32)
                assert tms[0] is not None and len(tms[0]) == 0
            else:
                tm_ref = oracle_mod.process_moving_object(frames[f - 1], frames[f])
                blur_ref, _ = oracle_mod.blur_flags(frames[f], boxes[f])
                if tm_ref is None:
                    assert tms[f] is None, f
                    tm_ref = np.zeros((0, 2), np.float32)
                else:
                    assert np.array_equal(tms[f], tm_ref), f
                    ntm_total += len(tm_ref)
            assert np.array_equal(flags[2 * f:2 * f + 2], blur_ref), f
            r = ex.extract(frames[f], boxes[f], tm_ref, blur_ref)
            for name in r["kps"].dtype.names:
                assert np.array_equal(out[f][0][name], r["kps"][name]), (f, name)
            assert np.array_equal(out[f][1], r["desc"]), f
        assert ntm_total > 0                       # the mask path is exercised
        assert all(n is None or n > 0 for n in nms)
    finally:
        bp.close()


def test_good_features_beyond_16384_maxima(ctx, oracle_mod):
    """A noise frame has more Harris local maxima than 16384: k_gf_select takes the sorted keys
    4096 at a time (radix select of each batch's lower bound), so the greedy selection stays the
    sequential one however many maxima there are -- the result equals the uncapped oracle, with
    maxCorners reached inside the first batch and, at minDistance 20 (fewer than 1000 corners fit),
    only after every batch; the whole ProcessMovingObject on such frames runs instead of failing."""
    rng = np.random.default_rng(11)
    noise = rng.integers(0, 256, (480, 640), dtype=np.uint8)
    with pytest.raises(RuntimeError):                 # the frame does exceed 16384 maxima
        oracle_mod.good_features(noise, max_cand=16384)
    ref = oracle_mod.good_features(noise)
    assert len(ref) == 1000
    eq(cf.GoodFeaturesToTrack(ctx, noise), ref, "noise")
    ref20 = oracle_mod.good_features(noise, min_distance=20.0)
    assert 0 < len(ref20) < 1000
    eq(cf.GoodFeaturesToTrack(ctx, noise, min_distance=20.0), ref20, "noise md20")
    cur = np.roll(noise, (1, 2), axis=(0, 1))
    tm = cf.ProcessMovingObject(ctx, noise, cur)
    tm_ref = oracle_mod.process_moving_object(noise, cur)
    if tm_ref is None:
        assert tm is None
    else:
        eq(tm, tm_ref, "noise T_M")
