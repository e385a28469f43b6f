"""The drop-in C++ adapters executed on the GPU (tests/adapter_shim/adapter_exec.cpp, built by
__graft_entry__.build()): ORB_SLAM2::ORBextractor::operator() (ORBextractor.h:73-75) on two
frames, coeb::SearchByProjectionLastFrame with the Tracking retry (Tracking.cc:947-958) and
coeb::PoseOptimization (Optimizer.cc:239-451), called from C++ with reference-shaped Frame /
MapPoint types, compared with the oracle.  Also the reference conventions the adapter keeps:
an empty image leaves the outputs untouched, no keypoints release the descriptors, and two
extractors with the same parameters share one pooled context, and an image larger than the
pooled context's 1280 x 960 (extracted on a worker thread) grows it instead of failing."""
import os
import subprocess

import numpy as np
import pytest

from coeb_front import KEYPOINT_DTYPE, make_camera, synth
from conftest import ROOT

pytestmark = pytest.mark.gpu
EXE = os.path.join(ROOT, "tests", "adapter_shim", "adapter_exec")


def test_adapters_run_against_library(tmp_path, oracle_mod):
    assert os.path.exists(EXE), "adapter_exec not built (run __graft_entry__.build())"
    W, H = 640, 480
    fr = synth.make_frames(W, H, 2, seed=4321)
    ex = oracle_mod.Extractor()
    r0, r1 = ex.extract(fr[0]), ex.extract(fr[1])
    depth = synth.make_depth(W, H)
    last = oracle_mod.mapframe_from_extraction(r0["kps"], r0["desc"], depth, synth.TUM_FX, synth.TUM_FY,
                                               synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
    ur, _ = oracle_mod.stereo_from_rgbd(r1["kps"], depth, synth.TUM_BF)
    Tc, Tl = synth.motion_pose(), np.eye(4, dtype=np.float32)
    cam = make_camera(synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF, W, H)
    d = str(tmp_path)

    def put(name, a):
        np.ascontiguousarray(a).tofile(os.path.join(d, name))
    put("size.i32", np.array([W, H], np.int32))
    put("frame0.u8", fr[0])
    put("frame1.u8", fr[1])
    put("cam.f32", np.array([cam.fx, cam.fy, cam.cx, cam.cy, cam.bf, cam.min_x, cam.max_x, cam.min_y, cam.max_y],
                            np.float32))
    put("Tc.f32", Tc.astype(np.float32))
    put("Tl.f32", Tl)
    put("last_has.u8", last["has_mp"].astype(np.uint8))
    put("last_nobs.i32", last["mp_nobs"].astype(np.int32))
    put("last_xw.f32", last["xw"].astype(np.float32))
    put("last_desc.u8", last["mp_desc"].astype(np.uint8))
    put("cur_ur.f32", ur.astype(np.float32))
    WB, HB = 1600, 1200                     # beyond the pooled context's initial 1280 x 960
    fb = synth.make_frames(WB, HB, 1, seed=99)[0]
    put("size_big.i32", np.array([WB, HB], np.int32))
    put("frame_big.u8", fb)
    out = subprocess.run([EXE, d], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr

    def get(name, dtype):
        return np.fromfile(os.path.join(d, name), dtype)
    for i, r in ((0, r0), (1, r1)):
        k = get("kps%d.bin" % i, np.uint8).view(KEYPOINT_DTYPE)
        desc = get("desc%d.u8" % i, np.uint8).reshape(-1, 32)
        assert len(k) == len(r["kps"]) > 900
        for f in KEYPOINT_DTYPE.names:
            assert np.array_equal(k[f], r["kps"][f]), (i, f)
        assert np.array_equal(desc, r["desc"]), i
    rb = oracle_mod.Extractor(2000, 1.2, 8, 20, 7).extract(fb)
    kb = get("kps_big.bin", np.uint8).view(KEYPOINT_DTYPE)
    assert len(kb) == len(rb["kps"]) > 1500
    for f in KEYPOINT_DTYPE.names:
        assert np.array_equal(kb[f], rb["kps"][f]), ("big", f)
    assert np.array_equal(get("desc_big.u8", np.uint8).reshape(-1, 32), rb["desc"])
    checks = dict(l.split() for l in open(os.path.join(d, "checks.txt")))
    assert checks == {"empty_untouched": "1", "flat_released": "1", "accessors": "1"}, checks
    # SearchByProjection with the retry of Tracking::TrackWithMotionModel
    cam_o = oracle_mod.camera(ex, W, H, synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
    nm_ref, m_ref = oracle_mod.search_by_projection(cam_o, r1["kps"], r1["desc"], ur, last, Tc, Tl, 15.0)
    if nm_ref < 20:
        nm_ref, m_ref = oracle_mod.search_by_projection(cam_o, r1["kps"], r1["desc"], ur, last, Tc, Tl, 30.0)
    assert int(get("nmatch.i32", np.int32)[0]) == nm_ref > 500
    assert np.array_equal(get("match.i32", np.int32), m_ref)
    # PoseOptimization on the matched frame, through the adapter
    has = (m_ref >= 0).astype(np.uint8)
    xw = np.zeros((len(m_ref), 3), np.float32)
    xw[m_ref >= 0] = last["xw"][m_ref[m_ref >= 0]]
    from coeb_front import Context
    c = Context(max_width=W, max_height=H, max_batch=1)
    isg = np.array(c.tables().inv_sigma2[:8], np.float32)        # mvInvLevelSigma2
    c.close()
    nin_ref, T_ref, o_ref = oracle_mod.pose_optimization(r1["kps"], has, xw, ur, isg, synth.TUM_FX, synth.TUM_FY,
                                                         synth.TUM_CX, synth.TUM_CY, synth.TUM_BF, Tc)
    assert int(get("pose_nin.i32", np.int32)[0]) == nin_ref > 0
    assert np.array_equal(get("pose_T.f32", np.float32).reshape(4, 4).view(np.uint32), T_ref.view(np.uint32))
    assert np.array_equal(get("pose_outl.u8", np.uint8)[has > 0], o_ref[has > 0])
