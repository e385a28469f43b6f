"""ctypes binding of oracle/liborb_oracle.so.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker / timed CPU baseline.  The product never imports it.
Parity vs the original reference binary: UNPINNED (see orb_oracle.h).
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liborb_oracle.so")

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
MAX_LEVELS = 16


class Params(C.Structure):
    _fields_ = [("nfeatures", C.c_int), ("scale_factor", C.c_double), ("nlevels", C.c_int),
                ("ini_th", C.c_int), ("min_th", C.c_int),
                ("scale", C.c_float * MAX_LEVELS), ("inv_scale", C.c_float * MAX_LEVELS),
                ("sigma2", C.c_float * MAX_LEVELS), ("inv_sigma2", C.c_float * MAX_LEVELS),
                ("nfeat", C.c_int * MAX_LEVELS), ("umax", C.c_int * 16),
                ("pattern", (C.c_int * 2) * 512)]


class Debug(C.Structure):
    _fields_ = [("pyramid", C.c_void_p), ("level_off", C.c_int64 * (MAX_LEVELS + 1)),
                ("ncand", C.c_int * MAX_LEVELS), ("nkept", C.c_int * MAX_LEVELS),
                ("area_flag", C.c_int)]


class Camera(C.Structure):
    _fields_ = [("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float),
                ("bf", C.c_float), ("mb", C.c_float),
                ("min_x", C.c_float), ("max_x", C.c_float), ("min_y", C.c_float), ("max_y", C.c_float),
                ("grid_inv_w", C.c_float), ("grid_inv_h", C.c_float),
                ("scale", C.c_float * MAX_LEVELS), ("nlevels", C.c_int)]


class LastFrame(C.Structure):
    _fields_ = [("n", C.c_int), ("has_mp", C.c_void_p), ("outlier", C.c_void_p), ("xw", C.c_void_p),
                ("mp_desc", C.c_void_p), ("mp_nobs", C.c_void_p), ("keys_un", C.c_void_p)]


class CurFrame(C.Structure):
    _fields_ = [("n", C.c_int), ("keys_un", C.c_void_p), ("desc", C.c_void_p), ("uright", C.c_void_p)]


class LocalMap(C.Structure):
    _fields_ = [("n", C.c_int), ("in_view", C.c_void_p), ("proj_x", C.c_void_p), ("proj_y", C.c_void_p),
                ("proj_xr", C.c_void_p), ("level", C.c_void_p), ("view_cos", C.c_void_p), ("desc", C.c_void_p),
                ("nobs", C.c_void_p)]


class KfPoints(C.Structure):
    _fields_ = [("n", C.c_int), ("valid", C.c_void_p), ("xw", C.c_void_p), ("desc", C.c_void_p),
                ("max_dist", C.c_void_p), ("min_dist", C.c_void_p), ("angle", C.c_void_p)]


KFPOINT_FIELDS = (("valid", np.uint8), ("world_pos", np.float32), ("descriptor", np.uint8),
                  ("max_distance", np.float32), ("min_distance", np.float32), ("angle", np.float32))


class Grid(C.Structure):
    _fields_ = [("cell_start", C.c_void_p), ("cell_idx", C.c_void_p)]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = C.CDLL(LIB)
        _lib.oc_fast_atan2.restype = C.c_float
        _lib.oc_fast_atan2.argtypes = [C.c_float, C.c_float]
        _lib.oc_sincos.argtypes = [C.c_float, C.c_void_p, C.c_void_p]
    return _lib


def ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


class Extractor:
    """ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST) on the CPU oracle."""

    def __init__(self, nfeatures=1000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7):
        self.p = Params()
        rc = lib().oc_init(C.byref(self.p), nfeatures, C.c_float(scale_factor), nlevels, ini_th, min_th)
        assert rc == 0

    @property
    def nlevels(self):
        return self.p.nlevels

    def level_sizes(self, w, h):
        out = []
        for l in range(self.p.nlevels):
            lw, lh = C.c_int(), C.c_int()
            lib().oc_level_size(C.byref(self.p), w, h, l, C.byref(lw), C.byref(lh))
            out.append((lw.value, lh.value))
        return out

    def extract(self, gray, boxes=None, tm=None, blur=None, debug=False):
        gray = np.ascontiguousarray(gray, dtype=np.uint8)
        h, w = gray.shape
        boxes = np.zeros((0, 4), np.float32) if boxes is None else np.ascontiguousarray(boxes, np.float32)
        tm = np.zeros((0, 2), np.float32) if tm is None else np.ascontiguousarray(tm, np.float32)
        blur = np.zeros(0, np.int32) if blur is None else np.ascontiguousarray(blur, np.int32)
        cap = 8 * self.p.nfeatures + 256
        kps = np.zeros(cap, KP_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = C.c_int()
        dbg = Debug()
        pyr = None
        if debug:
            total = sum(a * b for a, b in self.level_sizes(w, h))
            pyr = np.zeros(total, np.uint8)
            dbg.pyramid = pyr.ctypes.data
        rc = lib().oc_extract(C.byref(self.p), ptr(gray), w, h, w, ptr(boxes), len(boxes), ptr(tm), len(tm),
                              ptr(blur), len(blur), ptr(kps), ptr(desc), cap, C.byref(n), C.byref(dbg))
        if rc != 0:
            raise RuntimeError("oc_extract rc=%d" % rc)
        n = n.value
        res = dict(kps=kps[:n].copy(), desc=desc[:n].copy())
        if debug:
            res["pyramid"] = pyr
            res["level_off"] = list(dbg.level_off[: self.p.nlevels + 1])
            res["ncand"] = list(dbg.ncand[: self.p.nlevels])
            res["nkept"] = list(dbg.nkept[: self.p.nlevels])
            res["area_flag"] = dbg.area_flag
        return res


def camera(ex, w, h, fx, fy, cx, cy, bf):
    c = Camera()
    lib().oc_camera_init(C.byref(c), C.c_float(fx), C.c_float(fy), C.c_float(cx), C.c_float(cy),
                         C.c_float(bf), w, h, C.byref(ex.p))
    return c


def stereo_from_rgbd(kps, depth, bf):
    n = len(kps)
    ur = np.zeros(n, np.float32)
    dep = np.zeros(n, np.float32)
    depth = np.ascontiguousarray(depth, np.float32)
    lib().oc_stereo_from_rgbd(ptr(kps), n, ptr(depth), depth.shape[1], depth.shape[1], C.c_float(bf),
                              ptr(ur), ptr(dep))
    return ur, dep


def search_by_projection(cam, cur_kps, cur_desc, cur_ur, last, Tcw_cur, Tcw_last, th=15.0, bmono=False,
                         check_ori=True):
    """last: dict(has_mp u8[n], outlier u8[n], xw f32[n,3], mp_desc u8[n,32], mp_nobs i32[n], keys_un KP[n])"""
    cur_kps = np.ascontiguousarray(cur_kps)
    cur_desc = np.ascontiguousarray(cur_desc, np.uint8)
    cur_ur = np.ascontiguousarray(cur_ur, np.float32)
    cf = CurFrame(len(cur_kps), cur_kps.ctypes.data, cur_desc.ctypes.data, cur_ur.ctypes.data)
    arrs = {k: np.ascontiguousarray(v) for k, v in last.items()}
    lf = LastFrame(len(arrs["has_mp"]), arrs["has_mp"].ctypes.data, arrs["outlier"].ctypes.data,
                   arrs["xw"].ctypes.data, arrs["mp_desc"].ctypes.data, arrs["mp_nobs"].ctypes.data,
                   arrs["keys_un"].ctypes.data)
    out = np.zeros(max(len(cur_kps), 1), np.int32)
    Tc = np.ascontiguousarray(Tcw_cur, np.float32)
    Tl = np.ascontiguousarray(Tcw_last, np.float32)
    nm = lib().oc_search_by_projection(C.byref(cam), C.byref(cf), C.byref(lf), ptr(Tc), ptr(Tl),
                                       C.c_float(th), int(bmono), int(check_ori), ptr(out))
    return nm, out[: len(cur_kps)]


LOCALMAP_FIELDS = (("in_view", np.uint8), ("proj_x", np.float32), ("proj_y", np.float32), ("proj_xr", np.float32),
                   ("level", np.int32), ("view_cos", np.float32), ("descriptor", np.uint8), ("observations", np.int32))


def search_local_map(cam, cur_kps, cur_desc, cur_ur, cur_obs, mp, th=3.0, nnratio=0.8):
    """ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>, th) (ORBmatcher.cc:44-129).
    cur_obs: i32[n] Observations() of the MapPoint already on each current keypoint (-1: none).
    mp: dict of LOCALMAP_FIELDS arrays.  Returns (nmatches, match[n]: local-map index or -1)."""
    cur_kps = np.ascontiguousarray(cur_kps)
    cur_desc = np.ascontiguousarray(cur_desc, np.uint8)
    cur_ur = np.ascontiguousarray(cur_ur, np.float32)
    cur_obs = np.ascontiguousarray(cur_obs, np.int32)
    cf = CurFrame(len(cur_kps), cur_kps.ctypes.data, cur_desc.ctypes.data, cur_ur.ctypes.data)
    arrs = {k: np.ascontiguousarray(mp[k], dt) for k, dt in LOCALMAP_FIELDS}
    lm = LocalMap(len(arrs["in_view"]), *[arrs[k].ctypes.data for k, _ in LOCALMAP_FIELDS])
    out = np.zeros(max(len(cur_kps), 1), np.int32)
    nm = lib().oc_search_local_map(C.byref(cam), C.byref(cf), ptr(cur_obs), C.byref(lm), C.c_float(th),
                                   C.c_float(nnratio), ptr(out))
    return nm, out[: len(cur_kps)]


def search_keyframe(cam, cur_kps, cur_desc, cur_has, kf, Tcw, th=10.0, orb_dist=100, check_ori=True):
    """ORBmatcher::SearchByProjection(Frame&, KeyFrame*, set<MapPoint*>, th, ORBdist)
    (ORBmatcher.cc:1473-1560).  cur_has: u8[n], CurrentFrame.mvpMapPoints[i] != NULL at entry.
    kf: dict of KFPOINT_FIELDS arrays.  Returns (nmatches, match[n]: KeyFrame point index or -1)."""
    cur_kps = np.ascontiguousarray(cur_kps)
    cur_desc = np.ascontiguousarray(cur_desc, np.uint8)
    n = len(cur_kps)
    cur_has = np.zeros(n, np.uint8) if cur_has is None else np.ascontiguousarray(cur_has, np.uint8)
    dummy_ur = np.full(max(n, 1), -1, np.float32)
    cf = CurFrame(n, cur_kps.ctypes.data, cur_desc.ctypes.data, dummy_ur.ctypes.data)
    arrs = {k: np.ascontiguousarray(kf[k], dt) for k, dt in KFPOINT_FIELDS}
    kp = KfPoints(len(arrs["valid"]), *[arrs[k].ctypes.data for k, _ in KFPOINT_FIELDS])
    T = np.ascontiguousarray(Tcw, np.float32)
    out = np.zeros(max(n, 1), np.int32)
    nm = lib().oc_search_keyframe(C.byref(cam), C.byref(cf), ptr(cur_has), C.byref(kp), ptr(T), C.c_float(th),
                                  int(orb_dist), int(bool(check_ori)), ptr(out))
    return nm, out[:n]


class PoseFrame(C.Structure):
    _fields_ = [("n", C.c_int), ("has_mp", C.c_void_p), ("xw", C.c_void_p), ("keys_un", C.c_void_p),
                ("uright", C.c_void_p), ("inv_sigma2", C.c_void_p),
                ("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float), ("bf", C.c_float)]


def pose_optimization(kps, has_mp, xw, uright, inv_sigma2, fx, fy, cx, cy, bf, Tcw):
    """Optimizer::PoseOptimization(Frame*) (Optimizer.cc:239-451), canonical g2o LM.
    Returns (ninliers, Tcw_out[4,4] f32, outlier[n] u8 (0 where no MapPoint))."""
    kps = np.ascontiguousarray(kps)
    n = len(kps)
    has = np.ascontiguousarray(has_mp, np.uint8)
    xw = np.ascontiguousarray(xw, np.float32).reshape(n, 3) if n else np.zeros((1, 3), np.float32)
    ur = np.ascontiguousarray(uright, np.float32)
    isg = np.ascontiguousarray(inv_sigma2, np.float32)
    fr = PoseFrame(n, has.ctypes.data, xw.ctypes.data, kps.ctypes.data, ur.ctypes.data, isg.ctypes.data,
                   fx, fy, cx, cy, bf)
    T = np.ascontiguousarray(Tcw, np.float32).copy()
    out = np.zeros(max(n, 1), np.uint8)
    nin = lib().oc_pose_optimization(C.byref(fr), ptr(T), ptr(out))
    return nin, T.reshape(4, 4), out[:n]


class KfView(C.Structure):
    _fields_ = [("n", C.c_int), ("keys", C.c_void_p), ("has", C.c_void_p), ("xw", C.c_void_p)]


def local_map_build(cam, kf1, kf2, T_kf1_kf2, seen1, nobs, stride, Tcw_cur, cos_limit=0.5):
    """The batch chain's local map of a current frame (oc_local_map_build).
    kf1 / kf2: mapframe_from_extraction dicts of frames f-1 / f-2 (kf2 may be None).  Returns the
    LOCALMAP_FIELDS arrays over 2*stride slots ([0, stride) KF2, [stride, 2 stride) KF1) plus
    "xw" (2*stride, 3) world positions (valid where in view)."""
    M = 2 * stride
    arrs = {}
    views = []
    for kf in (kf1, kf2):
        if kf is None:
            views.append(None)
            continue
        keys = np.ascontiguousarray(kf["keys_un"])
        has = np.ascontiguousarray(kf["has_mp"], np.uint8)
        xw = np.ascontiguousarray(kf["xw"], np.float32)
        arrs[id(kf)] = (keys, has, xw)
        views.append(KfView(len(keys), keys.ctypes.data, has.ctypes.data, xw.ctypes.data))
    v1, v2 = views
    out = dict(in_view=np.zeros(M, np.uint8), proj_x=np.zeros(M, np.float32), proj_y=np.zeros(M, np.float32),
               proj_xr=np.zeros(M, np.float32), level=np.zeros(M, np.int32), view_cos=np.zeros(M, np.float32),
               observations=np.zeros(M, np.int32), xw=np.zeros((M, 3), np.float32))
    seen = np.zeros(stride, np.uint8) if seen1 is None else np.ascontiguousarray(seen1, np.uint8)
    T21 = np.ascontiguousarray(T_kf1_kf2 if T_kf1_kf2 is not None else np.eye(4), np.float32)
    Tc = np.ascontiguousarray(Tcw_cur, np.float32)
    nin = lib().oc_local_map_build(C.byref(cam), C.byref(v2) if v2 is not None else None, ptr(T21), C.byref(v1),
                                   ptr(seen), int(nobs), int(stride), ptr(Tc), C.c_float(cos_limit),
                                   ptr(out["in_view"]), ptr(out["proj_x"]), ptr(out["proj_y"]), ptr(out["proj_xr"]),
                                   ptr(out["level"]), ptr(out["view_cos"]), ptr(out["observations"]), ptr(out["xw"]))
    desc = np.zeros((M, 32), np.uint8)
    if kf2 is not None:
        desc[:len(kf2["mp_desc"])] = kf2["mp_desc"]
    desc[stride:stride + len(kf1["mp_desc"])] = kf1["mp_desc"]
    out["descriptor"] = desc
    out["n_in_view"] = nin
    return out


def track_frame(cam, isg, cur, ur, last, prev2, T_pred, T_last, stride, nobs=2, th=15.0, lth=3.0, nnratio=0.8,
                fx=0.0, fy=0.0, cx=0.0, cy=0.0, bf=0.0):
    """Tracking::Track for one RGB-D frame as the batch chain runs it (BASELINE configs[4]):
    TrackWithMotionModel (SearchByProjection th, retry 2 th below 20 matches, PoseOptimization,
    outlier discard, nmatchesMap >= 10; Tracking.cc:933-994) then TrackLocalMap (local map of
    KeyFrames f-1 = `last` and f-2 = `prev2`, SearchLocalPoints, PoseOptimization, inliers >= 30;
    :996-1047, 1222-1272).  last / prev2: mapframe_from_extraction dicts (world = last's camera;
    prev2 placed by T_last, frame f-1's pose relative to f-2).  cur: dict(kps, desc), ur its
    mvuRight.  Returns a dict of every intermediate result."""
    I4 = np.eye(4, dtype=np.float32)
    kps, desc = cur["kps"], cur["desc"]
    nm, m = search_by_projection(cam, kps, desc, ur, last, T_pred, I4, th)
    if nm < 20:
        nm, m = search_by_projection(cam, kps, desc, ur, last, T_pred, I4, 2 * th)
    res = dict(nmatches=nm, match=m, T1=np.asarray(T_pred, np.float32).copy(), nin1=0, nmatches_map=0,
               T=np.asarray(T_pred, np.float32).copy(), ninliers=0, nlocal=0, local_match=np.full(len(kps), -1, np.int32),
               state=0)
    if nm < 20:
        return res
    has = (m >= 0).astype(np.uint8)
    xw = np.zeros((len(m), 3), np.float32)
    xw[m >= 0] = last["xw"][m[m >= 0]]
    nin1, T1, o1 = pose_optimization(kps, has, xw, ur, isg, fx, fy, cx, cy, bf, T_pred)
    inlier = (has > 0) & (o1 == 0)
    nmap = int(inlier.sum()) if nobs > 0 else 0
    res.update(T1=T1, nin1=nin1, outlier1=o1, nmatches_map=nmap, T=T1.copy())
    if nmap < 10:
        return res
    seen = np.zeros(stride, np.uint8)
    seen[m[m >= 0]] = 1
    lm = local_map_build(cam, last, prev2, T_last, seen, nobs, stride, T1)
    cur_obs = np.where(inlier, nobs, -1).astype(np.int32)
    nl, lmatch = search_local_map(cam, kps, desc, ur, cur_obs, lm, lth, nnratio)
    has2 = ((lmatch >= 0) | inlier).astype(np.uint8)
    xw2 = np.where((lmatch >= 0)[:, None], lm["xw"][np.maximum(lmatch, 0)], xw).astype(np.float32)
    nin2, T2, o2 = pose_optimization(kps, has2, xw2, ur, isg, fx, fy, cx, cy, bf, T1)
    res.update(local_map=lm, nlocal=nl, local_match=lmatch, has2=has2, T=T2, ninliers=nin2, outlier=o2,
               state=2 if (nin2 if nobs > 0 else 0) >= 30 else 1)
    return res


def pose_last_stats():
    """(LM iterations, LM trials) of the last pose_optimization call on this thread."""
    it, tr = C.c_int(0), C.c_int(0)
    lib().oc_pose_last_stats(C.byref(it), C.byref(tr))
    return it.value, tr.value


def undistort_keypoints(kps, fx, fy, cx, cy, dist):
    """Frame::UndistortKeyPoints (Frame.cc:579-609); dist = (k1, k2, p1, p2, k3)."""
    kps = np.ascontiguousarray(kps)
    out = kps.copy()
    d = np.ascontiguousarray(np.asarray(dist, np.float32).reshape(5))
    lib().oc_undistort_keypoints(kps.ctypes.data_as(C.c_void_p), len(kps), C.c_float(fx), C.c_float(fy), C.c_float(cx),
                                 C.c_float(cy), ptr(d), out.ctypes.data_as(C.c_void_p))
    return out


def blur_flags(gray, boxes):
    gray = np.ascontiguousarray(gray, np.uint8)
    boxes = np.ascontiguousarray(boxes, np.float32)
    out = np.zeros(len(boxes), np.int32)
    mean = np.zeros(len(boxes), np.float64)
    h, w = gray.shape
    lib().oc_blur_flags(ptr(gray), w, h, w, ptr(boxes), len(boxes), ptr(out), ptr(mean))
    return out, mean


def descriptor_distance(a, b):
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    return lib().oc_descriptor_distance(ptr(a), ptr(b))


def fast_atan2(y, x):
    return lib().oc_fast_atan2(C.c_float(y), C.c_float(x))


def sincos(a):
    s, c = C.c_float(), C.c_float()
    lib().oc_sincos(C.c_float(a), C.byref(s), C.byref(c))
    return s.value, c.value


def gaussian_blur7(img):
    """GaussianBlur(7x7, sigma 2, REFLECT_101) of one pyramid level (ORBextractor.cc:1317-1318)."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    out = np.zeros_like(img)
    lib().oc_gaussian_blur7(ptr(img), w, h, w, ptr(out), w)
    return out


def gauss_kernel7():
    k = (C.c_int * 7)()
    lib().oc_gauss_kernel7(k)
    return list(k)


def image_to_gray(img, rgb_order=1):
    """Tracking::GrabImageRGBD gray conversion (Tracking.cc:212-225): (h, w) gray, (h, w, 3) or
    (h, w, 4) images."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape[:2]
    ch = 1 if img.ndim == 2 else img.shape[2]
    out = np.zeros((h, w), np.uint8)
    lib().oc_image_to_gray(ptr(img), w, h, ch * w, ch, rgb_order, ptr(out))
    return out


def depth_to_float(depth, factor):
    """Tracking.cc:227-228: uint16 or float32 depth map -> float32 (convertTo with mDepthMapFactor;
    a float32 map with factor 1 is returned unchanged)."""
    depth = np.ascontiguousarray(depth)
    h, w = depth.shape
    dt = {np.dtype(np.uint16): 0, np.dtype(np.float32): 1}[depth.dtype]
    out = np.zeros((h, w), np.float32)
    lib().oc_depth_to_float(ptr(depth), w, h, C.c_size_t(depth.strides[0]), dt, C.c_float(factor), ptr(out))
    return out


def rgb2gray(rgb, rgb_order=1):
    rgb = np.ascontiguousarray(rgb, np.uint8)
    h, w, _ = rgb.shape
    out = np.zeros((h, w), np.uint8)
    lib().oc_rgb2gray(ptr(rgb), w, h, 3 * w, rgb_order, ptr(out))
    return out


def mapframe_from_extraction(kps, desc, depth, cam_fx, cam_fy, cam_cx, cam_cy, bf, nobs=2):
    """LastFrame snapshot from an extracted frame with Tcw = I: MapPoint = UnprojectStereo(i)
    (src/Frame.cc:844-858) for every keypoint with depth > 0, descriptor = its own."""
    ur, dep = stereo_from_rgbd(kps, depth, bf)
    n = len(kps)
    has = (dep > 0).astype(np.uint8)
    z = dep.astype(np.float32)
    invfx = np.float32(1.0) / np.float32(cam_fx)
    invfy = np.float32(1.0) / np.float32(cam_fy)
    u = kps["x"].astype(np.float32)
    v = kps["y"].astype(np.float32)
    x = ((u - np.float32(cam_cx)) * z) * invfx
    y = ((v - np.float32(cam_cy)) * z) * invfy
    xw = np.stack([x, y, z], axis=1).astype(np.float32)
    return dict(has_mp=has, outlier=np.zeros(n, np.uint8), xw=np.ascontiguousarray(xw),
                mp_desc=np.ascontiguousarray(desc, np.uint8), mp_nobs=np.full(n, nobs, np.int32),
                keys_un=np.ascontiguousarray(kps))


# ---- Frame::ProcessMovingObject (Frame.cc:311-393) ----
def _gray(img):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    return img, img.shape[1], img.shape[0]


def good_features(img, max_corners=1000, quality=0.01, min_distance=8.0, k=0.04, max_cand=1 << 30):
    """cv::goodFeaturesToTrack(img, .., maxCorners, quality, minDistance, Mat(), 3, true, k): (n, 2) f32."""
    img, w, h = _gray(img)
    out = np.zeros((max(max_corners, 1), 2), np.float32)
    n = lib().oc_good_features_harris(ptr(img), w, h, w, max_corners, C.c_double(quality), C.c_double(min_distance),
                                      C.c_double(k), ptr(out), len(out), max_cand)
    if n < 0:
        raise RuntimeError("goodFeaturesToTrack oracle: candidate cap exceeded")
    return out[:min(n, len(out))].copy()


def corner_subpix(img, xy, win=10, max_iter=20, eps=0.03):
    """cv::cornerSubPix(img, xy, Size(win, win), Size(-1,-1), TermCriteria(ITER|EPS, max_iter, eps))."""
    img, w, h = _gray(img)
    xy = np.ascontiguousarray(xy, dtype=np.float32).copy()
    lib().oc_corner_subpix(ptr(img), w, h, w, ptr(xy), len(xy), win, max_iter, C.c_double(eps))
    return xy


def lk_pyr(prev, nxt, xy, win=22, max_level=5, max_count=20, eps=0.01):
    """cv::calcOpticalFlowPyrLK(prev, next, xy, ..., Size(win, win), max_level, (ITER|EPS, max_count, eps)):
    (next_xy (n,2) f32, status (n,) u8)."""
    prev, w, h = _gray(prev)
    nxt = np.ascontiguousarray(nxt, dtype=np.uint8)
    xy = np.ascontiguousarray(xy, dtype=np.float32)
    out = np.zeros_like(xy)
    st = np.zeros(len(xy), np.uint8)
    lib().oc_lk_pyr(ptr(prev), ptr(nxt), w, h, w, ptr(xy), len(xy), win, max_level, max_count, C.c_double(eps),
                    ptr(out), ptr(st))
    return out, st


def pyr_down(img):
    img, w, h = _gray(img)
    out = np.zeros(((h + 1) // 2, (w + 1) // 2), np.uint8)
    lib().oc_pyr_down(ptr(img), w, h, ptr(out))
    return out


def find_fundamental(m1, m2, thr=0.1, conf=0.99):
    """cv::findFundamentalMat(m1, m2, mask, FM_RANSAC, thr, conf): 3x3 f64 or None (empty Mat)."""
    m1 = np.ascontiguousarray(m1, dtype=np.float32)
    m2 = np.ascontiguousarray(m2, dtype=np.float32)
    F = np.zeros(9, np.float64)
    ok = lib().oc_find_fundamental(ptr(m1), ptr(m2), len(m1), C.c_double(thr), C.c_double(conf), ptr(F))
    return F.reshape(3, 3) if ok else None


def moving_tail(prev, cur, pxy, nxy, state, edge=5, limit=2120.0):
    """SAD check + findFundamentalMat + epipolar distance (Frame.cc:337-384) on tracked pairs:
    (T_M (m,2) f32 or None when F is empty, state after the SAD check, F or None, |F_ sets|)."""
    prev, w, h = _gray(prev)
    cur = np.ascontiguousarray(cur, dtype=np.uint8)
    pxy = np.ascontiguousarray(pxy, dtype=np.float32)
    nxy = np.ascontiguousarray(nxy, dtype=np.float32)
    st = np.ascontiguousarray(state, dtype=np.uint8).copy()
    tm = np.zeros((max(len(pxy), 1), 2), np.float32)
    F = np.zeros(9, np.float64)
    nf = C.c_int(0)
    nt = lib().oc_moving_tail(ptr(prev), ptr(cur), w, h, w, ptr(pxy), ptr(nxy), ptr(st), len(pxy), edge,
                              C.c_double(limit), ptr(tm), len(tm), ptr(F), C.byref(nf))
    if nt < 0:
        return None, st, None, nf.value
    return tm[:nt].copy(), st, F.reshape(3, 3), nf.value


def process_moving_object(prev, cur):
    """Frame::ProcessMovingObject(imgray, box) with imGrayPre = prev: T_M (m,2) f32, or None
    when findFundamentalMat returns an empty Mat."""
    prev, w, h = _gray(prev)
    cur = np.ascontiguousarray(cur, dtype=np.uint8)
    tm = np.zeros((1000, 2), np.float32)
    nc = C.c_int(0)
    nt = lib().oc_process_moving_object(ptr(prev), ptr(cur), w, h, w, ptr(tm), len(tm), C.byref(nc))
    return None if nt < 0 else tm[:nt].copy()


def fd_math(name, x):
    """canonical double acos / log / exp / cos"""
    f = getattr(lib(), "oc_fd_" + name)
    f.restype = C.c_double
    f.argtypes = [C.c_double]
    return f(x)


def solve_cubic(c):
    c = np.ascontiguousarray(c, dtype=np.float64)
    r = np.zeros(3, np.float64)
    n = lib().oc_solve_cubic(ptr(c), ptr(r))
    return n, r
