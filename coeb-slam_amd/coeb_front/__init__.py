"""Python mirror of the reference's front-end interface over the C-ABI (include/coeb_front.h).

  ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)
      include/ORBextractor.h:50-51; __call__ mirrors operator() (ORBextractor.h:73-75,
      src/ORBextractor.cc:1088-1342) and returns (keypoints, descriptors) instead of filling
      output arguments.  Accessors GetLevels/GetScaleFactor/... as ORBextractor.h:77-99.
  ORBmatcher(nnratio=0.6, checkOri=True).SearchByProjection(CurrentFrame, LastFrame, th, bMono)
      include/ORBmatcher.h:41,52, src/ORBmatcher.cc:1329-1471; mutates
      CurrentFrame.mvpMapPoints (slot index of the LastFrame MapPoint, -1 = NULL) and returns
      nmatches.
  ORBmatcher(nnratio).SearchByProjection(F, LocalMap, th=3)
      include/ORBmatcher.h:46, src/ORBmatcher.cc:44-129 (the Tracking::SearchLocalPoints call,
      src/Tracking.cc:1222-1271); assigns F.mvpMapPoints[i] = local-map index and returns nmatches.
  ORBmatcher(nnratio, checkOri).SearchByProjection(F, KeyFramePoints, sAlreadyFound, th, ORBdist)
      include/ORBmatcher.h:55, src/ORBmatcher.cc:1473-1600 (Tracking::Relocalization,
      src/Tracking.cc:1531,1545); assigns F.mvpMapPoints[i] = KeyFrame point index.
  ORBmatcher.DescriptorDistance(a, b)  src/ORBmatcher.cc:1648-1664
  Optimizer.PoseOptimization(F, camera)  include/Optimizer.h:47, src/Optimizer.cc:239-451; reads
      F.mvpMapPoints (>= 0: has a MapPoint) and F.mvMapPointPos, sets F.mTcw and F.mvbOutlier.

All compute runs in libcoeb_front.so (hand-written gfx950 HIP kernels).  There is no CPU
fallback: importing works anywhere, but constructing an extractor without the built library
or without a gfx950 device raises.
"""
import ctypes as C
import os
import re

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# COEB_LIB_PATH: an alternative build of the same library (kernel experiments); never a fallback
LIB_PATH = os.environ.get("COEB_LIB_PATH") or os.path.join(os.path.dirname(HERE), "lib", "libcoeb_front.so")

KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
assert KEYPOINT_DTYPE.itemsize == 28
MAX_LEVELS = 16
DEPTH_U16, DEPTH_F32 = 0, 1          # COEB_DEPTH_U16 / COEB_DEPTH_F32

# exported symbols of include/coeb_front.h (checked by tests/test_capi_symbols.py)
ABI_SYMBOLS = [
    "coeb_abi_version", "coeb_create", "coeb_destroy", "coeb_last_error", "coeb_orb_tables_get", "coeb_max_keypoints",
    "coeb_extract", "coeb_extract_batch_device", "coeb_batch_results", "coeb_match_batch_device",
    "coeb_match_batch_device_tcw",
    "coeb_batch_match_results", "coeb_match_lastframe", "coeb_blur_flags", "coeb_stereo_from_rgbd",
    "coeb_rgbd_preprocess", "coeb_descriptor_distance", "coeb_profile_enable", "coeb_profile_read",
    "coeb_profile_reset", "coeb_synchronize", "coeb_device_count", "coeb_debug_read",
    "coeb_device_alloc", "coeb_device_free", "coeb_memcpy_h2d", "coeb_memcpy_d2h", "coeb_set_batch_streams",
    "coeb_match_localmap", "coeb_match_keyframe", "coeb_pose_optimization", "coeb_undistort_keypoints",
    "coeb_boxes_from_int64", "coeb_good_features", "coeb_corner_subpix", "coeb_optical_flow_pyr_lk",
    "coeb_moving_tail", "coeb_moving_object_points", "coeb_moving_object_points_device",
    "coeb_pose_batch_device", "coeb_batch_pose_results",
    "coeb_host_alloc", "coeb_host_free", "coeb_memcpy_h2d_async", "coeb_memcpy_d2h_async",
    "coeb_copyq_create", "coeb_copyq_destroy", "coeb_copyq_h2d", "coeb_copyq_d2h", "coeb_copyq_after_ctx",
    "coeb_ctx_after_copyq", "coeb_copyq_synchronize", "coeb_frame_batch_device", "coeb_batch_frame_results",
    "coeb_track_local_map_batch_device", "coeb_batch_track_results", "coeb_rgbd_preprocess_batch_device",
    "coeb_marker_create", "coeb_marker_destroy", "coeb_marker_record_ctx", "coeb_marker_record_copyq",
    "coeb_ctx_wait_marker", "coeb_copyq_wait_marker", "coeb_marker_synchronize",
    "coeb_tum_read_list", "coeb_tum_associate",
]
# COEB_ABI_VERSION of the include/coeb_front.h these argtypes are written against; lib() refuses
# a library that reports another (tests/test_capi_symbols.py keeps the two equal)
ABI_VERSION = 3


class OrbParams(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("ini_th_fast", C.c_int32), ("min_th_fast", C.c_int32)]


class OrbTables(C.Structure):
    _fields_ = [("nlevels", C.c_int32), ("scale_factor", C.c_float),
                ("scale", C.c_float * MAX_LEVELS), ("inv_scale", C.c_float * MAX_LEVELS),
                ("sigma2", C.c_float * MAX_LEVELS), ("inv_sigma2", C.c_float * MAX_LEVELS),
                ("features_per_level", C.c_int32 * MAX_LEVELS), ("umax", C.c_int32 * 16)]


class Camera(C.Structure):
    _fields_ = [("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float), ("bf", C.c_float),
                ("min_x", C.c_float), ("max_x", C.c_float), ("min_y", C.c_float), ("max_y", C.c_float)]


class LastFrameC(C.Structure):
    _fields_ = [("n", C.c_int32), ("has_mappoint", C.c_void_p), ("outlier", C.c_void_p), ("world_pos", C.c_void_p),
                ("mp_descriptor", C.c_void_p), ("mp_observations", C.c_void_p), ("keys_un", C.c_void_p)]


class CurFrameC(C.Structure):
    _fields_ = [("n", C.c_int32), ("keys_un", C.c_void_p), ("descriptors", C.c_void_p), ("u_right", C.c_void_p)]


class LocalMapC(C.Structure):
    _fields_ = [("n", C.c_int32), ("in_view", C.c_void_p), ("proj_x", C.c_void_p), ("proj_y", C.c_void_p),
                ("proj_xr", C.c_void_p), ("level", C.c_void_p), ("view_cos", C.c_void_p), ("descriptor", C.c_void_p),
                ("observations", C.c_void_p)]


class KeyFramePointsC(C.Structure):
    _fields_ = [("n", C.c_int32), ("valid", C.c_void_p), ("world_pos", C.c_void_p), ("descriptor", C.c_void_p),
                ("max_distance", C.c_void_p), ("min_distance", C.c_void_p), ("angle", C.c_void_p)]


class PoseFrameC(C.Structure):
    _fields_ = [("n", C.c_int32), ("has_mappoint", C.c_void_p), ("world_pos", C.c_void_p), ("keys_un", C.c_void_p),
                ("u_right", C.c_void_p)]


class CoebError(RuntimeError):
    pass


_lib = None


def lib():
    """Load libcoeb_front.so (in-tree build); raise if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise CoebError("libcoeb_front.so not built (run __graft_entry__.build() or make -C coeb-slam_amd/csrc)")
        L = C.CDLL(LIB_PATH)
        got = L.coeb_abi_version()
        if got != ABI_VERSION:
            raise CoebError("%s reports ABI %d, this binding is written for ABI %d (rebuild the library)"
                            % (LIB_PATH, got, ABI_VERSION))
        L.coeb_create.restype = C.c_void_p
        L.coeb_create.argtypes = [C.POINTER(OrbParams), C.c_int, C.c_int, C.c_int, C.c_int]
        L.coeb_destroy.argtypes = [C.c_void_p]
        L.coeb_last_error.restype = C.c_char_p
        L.coeb_last_error.argtypes = [C.c_void_p]
        L.coeb_orb_tables_get.argtypes = [C.c_void_p, C.POINTER(OrbTables)]
        L.coeb_max_keypoints.argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.coeb_extract.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_size_t, C.c_void_p, C.c_int,
                                   C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int,
                                   C.POINTER(C.c_int)]
        L.coeb_extract_batch_device.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                                C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.coeb_frame_batch_device.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                              C.c_void_p]
        L.coeb_batch_frame_results.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                               C.POINTER(C.c_int), C.POINTER(C.c_void_p)]
        L.coeb_batch_results.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                         C.POINTER(C.c_void_p), C.POINTER(C.c_int)]
        L.coeb_match_batch_device.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(Camera),
                                              C.c_void_p, C.c_float, C.c_int32]
        L.coeb_match_batch_device_tcw.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                                  C.POINTER(Camera), C.c_void_p, C.c_float, C.c_int32]
        L.coeb_batch_match_results.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]
        L.coeb_pose_batch_device.argtypes = [C.c_void_p, C.POINTER(Camera), C.c_int, C.c_void_p, C.c_int32]
        L.coeb_batch_pose_results.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                              C.POINTER(C.c_void_p)]
        L.coeb_track_local_map_batch_device.argtypes = [C.c_void_p, C.POINTER(Camera), C.c_int, C.c_int32, C.c_float,
                                                        C.c_float]
        L.coeb_batch_track_results.argtypes = [C.c_void_p] + [C.POINTER(C.c_void_p)] * 6
        L.coeb_rgbd_preprocess_batch_device.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int,
                                                        C.c_float, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        L.coeb_match_lastframe.argtypes = [C.c_void_p, C.POINTER(Camera), C.POINTER(CurFrameC),
                                           C.POINTER(LastFrameC), C.c_void_p, C.c_void_p, C.c_float, C.c_int,
                                           C.c_int, C.c_void_p, C.POINTER(C.c_int)]
        L.coeb_match_localmap.argtypes = [C.c_void_p, C.POINTER(Camera), C.POINTER(CurFrameC), C.c_void_p,
                                          C.POINTER(LocalMapC), C.c_float, C.c_float, C.c_void_p, C.POINTER(C.c_int)]
        L.coeb_match_keyframe.argtypes = [C.c_void_p, C.POINTER(Camera), C.POINTER(CurFrameC), C.c_void_p,
                                          C.POINTER(KeyFramePointsC), C.c_void_p, C.c_float, C.c_int, C.c_int,
                                          C.c_void_p, C.POINTER(C.c_int)]
        L.coeb_pose_optimization.argtypes = [C.c_void_p, C.POINTER(Camera), C.POINTER(PoseFrameC), C.c_void_p,
                                             C.c_void_p, C.POINTER(C.c_int)]
        L.coeb_undistort_keypoints.argtypes = [C.c_void_p, C.POINTER(Camera), C.c_void_p, C.c_void_p, C.c_int,
                                               C.c_void_p]
        L.coeb_boxes_from_int64.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        L.coeb_good_features.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_size_t, C.c_int, C.c_double,
                                         C.c_double, C.c_double, C.c_void_p, C.c_int, C.POINTER(C.c_int)]
        L.coeb_corner_subpix.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_size_t, C.c_void_p, C.c_int,
                                         C.c_int, C.c_int, C.c_double]
        L.coeb_optical_flow_pyr_lk.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_size_t,
                                               C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double,
                                               C.c_void_p, C.c_void_p]
        L.coeb_moving_tail.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_size_t, C.c_void_p,
                                       C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_int),
                                       C.c_void_p, C.POINTER(C.c_int)]
        L.coeb_moving_object_points.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_size_t,
                                                C.c_void_p, C.c_int, C.POINTER(C.c_int), C.c_void_p]
        L.coeb_moving_object_points_device.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                                                       C.c_size_t, C.c_void_p, C.c_int, C.POINTER(C.c_int),
                                                       C.c_void_p]
        L.coeb_blur_flags.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_size_t, C.c_void_p, C.c_int,
                                      C.c_void_p]
        L.coeb_stereo_from_rgbd.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int,
                                            C.c_size_t, C.c_float, C.c_void_p, C.c_void_p]
        L.coeb_rgbd_preprocess.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_void_p,
                                           C.c_size_t, C.c_int, C.c_float, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        L.coeb_descriptor_distance.argtypes = [C.c_void_p, C.c_void_p]
        L.coeb_tum_read_list.argtypes = [C.c_char_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                         C.POINTER(C.c_int)]
        L.coeb_tum_associate.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_double, C.c_double,
                                         C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_int)]
        L.coeb_profile_enable.argtypes = [C.c_void_p, C.c_int]
        L.coeb_profile_reset.argtypes = [C.c_void_p]
        L.coeb_profile_read.argtypes = [C.c_void_p, C.c_char_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int,
                                        C.POINTER(C.c_int)]
        L.coeb_synchronize.argtypes = [C.c_void_p]
        L.coeb_set_batch_streams.argtypes = [C.c_void_p, C.c_int]
        L.coeb_device_alloc.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(C.c_void_p)]
        L.coeb_device_free.argtypes = [C.c_void_p, C.c_void_p]
        L.coeb_memcpy_h2d.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
        L.coeb_memcpy_d2h.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
        L.coeb_host_alloc.argtypes = [C.c_size_t, C.POINTER(C.c_void_p)]
        L.coeb_host_free.argtypes = [C.c_void_p]
        L.coeb_memcpy_h2d_async.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
        L.coeb_memcpy_d2h_async.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
        L.coeb_copyq_create.restype = C.c_void_p
        L.coeb_copyq_create.argtypes = [C.c_void_p]
        L.coeb_copyq_destroy.argtypes = [C.c_void_p]
        L.coeb_copyq_h2d.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
        L.coeb_copyq_d2h.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
        L.coeb_copyq_after_ctx.argtypes = [C.c_void_p, C.c_void_p]
        L.coeb_ctx_after_copyq.argtypes = [C.c_void_p, C.c_void_p]
        L.coeb_copyq_synchronize.argtypes = [C.c_void_p]
        L.coeb_marker_create.restype = C.c_void_p
        L.coeb_marker_create.argtypes = [C.c_void_p]
        for nm in ("coeb_marker_destroy", "coeb_marker_synchronize"):
            getattr(L, nm).argtypes = [C.c_void_p]
        for nm in ("coeb_marker_record_ctx", "coeb_marker_record_copyq", "coeb_ctx_wait_marker",
                   "coeb_copyq_wait_marker"):
            getattr(L, nm).argtypes = [C.c_void_p, C.c_void_p]
        L.coeb_debug_read.argtypes = [C.c_void_p, C.c_char_p, C.c_int, C.c_void_p, C.c_size_t,
                                      C.POINTER(C.c_size_t)]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


class Context:
    """One coeb_ctx: device buffers + HIP stream of one host thread (not reentrant)."""

    def __init__(self, nfeatures=1000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7, device=0,
                 max_width=1280, max_height=960, max_batch=1):
        L = lib()
        self.params = OrbParams(nfeatures, scale_factor, nlevels, ini_th, min_th)
        h = L.coeb_create(C.byref(self.params), device, max_width, max_height, max_batch)
        if not h:
            raise CoebError(L.coeb_last_error(None).decode())
        self.h = C.c_void_p(h)
        self.device = device

    def close(self):
        if getattr(self, "h", None):
            lib().coeb_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, rc):
        if rc != 0:
            raise CoebError("coeb rc=%d: %s" % (rc, lib().coeb_last_error(self.h).decode()))
        return rc

    def tables(self):
        t = OrbTables()
        self.check(lib().coeb_orb_tables_get(self.h, C.byref(t)))
        return t

    def max_keypoints(self, w, h):
        cache = self.__dict__.setdefault("_kcap", {})
        r = cache.get((w, h))
        if r is None:
            r = lib().coeb_max_keypoints(self.h, w, h)
            if r < 0:
                self.check(r)
            cache[(w, h)] = r
        return r

    # ---- single frame (host buffers) ----
    def extract(self, gray, boxes=None, tm=None, blur=None):
        gray = np.ascontiguousarray(gray, np.uint8)
        if gray.size == 0:
            return np.zeros(0, KEYPOINT_DTYPE), None
        h, w = gray.shape
        boxes = None if boxes is None else np.ascontiguousarray(boxes, np.float32)
        tm = None if tm is None else np.ascontiguousarray(tm, np.float32)
        blur = None if blur is None else np.ascontiguousarray(blur, np.int32)
        nb = 0 if boxes is None else len(boxes)
        nt = 0 if tm is None else len(tm)
        nf = 0 if blur is None else len(blur)
        cap = self.max_keypoints(w, h)
        # outputs written by the call (no zero fill) and returned as their first n rows (no copy):
        # the per-call cost of the binding is part of the drop-in latency bench.py measures
        kps = np.empty(cap, KEYPOINT_DTYPE)
        desc = np.empty((cap, 32), np.uint8)
        n = C.c_int()
        self.check(lib().coeb_extract(self.h, _p(gray), w, h, w, _p(boxes) if nb else None, nb,
                                      _p(tm) if nt else None, nt, _p(blur) if nf else None,
                                      nf, _p(kps), _p(desc), cap, C.byref(n)))
        n = n.value
        return kps[:n], (desc[:n] if n else None)

    # ---- device-resident batch ----
    def extract_batch_device(self, d_gray_ptr, nframes, w, h, boxes=None, box_off=None, tm=None, tm_off=None,
                             blur=None):
        args = []
        keep = []
        for a, dt in ((boxes, np.float32), (box_off, np.int32), (tm, np.float32), (tm_off, np.int32),
                      (blur, np.int32)):
            if a is None:
                args.append(None)
            else:
                a = np.ascontiguousarray(a, dt)
                keep.append(a)
                args.append(_p(a))
        self.check(lib().coeb_extract_batch_device(self.h, C.c_void_p(d_gray_ptr), nframes, w, h, *args))

    def frame_batch_device(self, d_gray_ptr, nframes, w, h, boxes=None, box_off=None):
        """The RGB-D Frame constructor on the batch (coeb_frame_batch_device): T_M from the previous
        frame, box blur flags and the masked extraction, all on the device."""
        b = None if boxes is None else np.ascontiguousarray(boxes, np.float32)
        o = None if box_off is None else np.ascontiguousarray(box_off, np.int32)
        self.check(lib().coeb_frame_batch_device(self.h, C.c_void_p(d_gray_ptr), nframes, w, h, _p(b), _p(o)))

    def batch_frame_results(self, nframes, nbox=0):
        """Host copies of the last frame batch's T_M (list of (n, 2) arrays, None where F was
        empty) and blur flags (nbox,)."""
        tm, ntm, cap, blur = C.c_void_p(), C.c_void_p(), C.c_int(), C.c_void_p()
        self.check(lib().coeb_batch_frame_results(self.h, C.byref(tm), C.byref(ntm), C.byref(cap), C.byref(blur)))
        n = self.download(ntm.value, 4 * nframes, np.int32)
        pts = self.download(tm.value, 8 * cap.value * nframes, np.float32).reshape(nframes, cap.value, 2)
        tms = [None if n[f] < 0 else pts[f, :n[f]].copy() for f in range(nframes)]
        flags = self.download(blur.value, 4 * nbox, np.int32) if nbox and blur.value else np.zeros(0, np.int32)
        return tms, flags

    def batch_results(self):
        k, d, n = C.c_void_p(), C.c_void_p(), C.c_void_p()
        cap = C.c_int()
        self.check(lib().coeb_batch_results(self.h, C.byref(k), C.byref(d), C.byref(n), C.byref(cap)))
        return k.value, d.value, n.value, cap.value

    def match_batch_device(self, d_depth_ptr, nframes, w, h, cam, Tcw, th=15.0, nobs=2):
        Tcw = np.ascontiguousarray(Tcw, np.float32)
        self.check(lib().coeb_match_batch_device(self.h, C.c_void_p(d_depth_ptr), nframes, w, h, C.byref(cam),
                                                 _p(Tcw), th, nobs))

    def match_batch_device_tcw(self, d_depth_ptr, nframes, w, h, cam, d_tcw_ptr, th=15.0, nobs=2):
        """As match_batch_device, with the (nframes, 4, 4) poses already in device memory."""
        self.check(lib().coeb_match_batch_device_tcw(self.h, C.c_void_p(d_depth_ptr), nframes, w, h, C.byref(cam),
                                                     C.c_void_p(d_tcw_ptr), th, nobs))

    def batch_match_results(self):
        m, n = C.c_void_p(), C.c_void_p()
        self.check(lib().coeb_batch_match_results(self.h, C.byref(m), C.byref(n)))
        return m.value, n.value

    def pose_batch_device(self, cam, nframes, d_tcw_ptr, min_matches=20):
        """TrackWithMotionModel's PoseOptimization over the batch matched last (Tracking.cc:947-964)."""
        self.check(lib().coeb_pose_batch_device(self.h, C.byref(cam), nframes, C.c_void_p(d_tcw_ptr), min_matches))

    def batch_pose_results(self):
        t, n, o = C.c_void_p(), C.c_void_p(), C.c_void_p()
        self.check(lib().coeb_batch_pose_results(self.h, C.byref(t), C.byref(n), C.byref(o)))
        return t.value, n.value, o.value

    def track_local_map_batch_device(self, cam, nframes, nkf=2, th=3.0, nnratio=0.8):
        """Tracking::TrackLocalMap over the batch posed last (coeb_track_local_map_batch_device):
        outlier discard, local map of KeyFrames f-1 / f-2 through isInFrustum, the local-map
        SearchByProjection(th = 3 for RGB-D, Tracking.cc:1264-1270), second PoseOptimization."""
        self.check(lib().coeb_track_local_map_batch_device(self.h, C.byref(cam), nframes, int(nkf), float(th),
                                                           float(nnratio)))

    def rgbd_preprocess_batch_device(self, d_img, channels, rgb_order, d_depth, depth_type, depth_scale, nframes, w, h,
                                     d_gray, d_depth_out):
        """GrabImageRGBD's cvtColor + depth convertTo over a packed device batch."""
        self.check(lib().coeb_rgbd_preprocess_batch_device(self.h, C.c_void_p(d_img), channels, rgb_order,
                                                           C.c_void_p(d_depth), depth_type, float(depth_scale), nframes,
                                                           w, h, C.c_void_p(d_gray), C.c_void_p(d_depth_out)))

    def batch_track_results(self):
        """Device pointers (Tcw, ninliers, nmatches_map, nlocal, local_match, outlier)."""
        ps = [C.c_void_p() for _ in range(6)]
        self.check(lib().coeb_batch_track_results(self.h, *[C.byref(p) for p in ps]))
        return tuple(p.value for p in ps)

    def synchronize(self):
        self.check(lib().coeb_synchronize(self.h))

    def set_batch_streams(self, n):
        """HIP streams a batch is chunked over (1 = serial on the context stream)."""
        self.check(lib().coeb_set_batch_streams(self.h, int(n)))

    def debug_read(self, what, f=0):
        size = C.c_size_t()
        self.check(lib().coeb_debug_read(self.h, what.encode(), f, None, 0, C.byref(size)))
        buf = np.zeros(size.value, np.uint8)
        self.check(lib().coeb_debug_read(self.h, what.encode(), f, _p(buf), size.value, C.byref(size)))
        return buf

    # ---- caller-owned device buffers ----
    def alloc(self, nbytes):
        return DeviceBuffer(self, nbytes)

    def upload(self, arr):
        arr = np.ascontiguousarray(arr)
        buf = DeviceBuffer(self, arr.nbytes)
        buf.write(arr)
        return buf

    def download(self, dptr, nbytes, dtype=np.uint8):
        out = np.empty(nbytes // np.dtype(dtype).itemsize, dtype)
        if nbytes:
            self.check(lib().coeb_memcpy_d2h(self.h, _p(out), C.c_void_p(dptr), nbytes))
        return out

    def download_into(self, dptr, out):
        """Copy out.nbytes bytes from device pointer dptr into the contiguous array out."""
        assert out.flags["C_CONTIGUOUS"]
        if out.nbytes:
            self.check(lib().coeb_memcpy_d2h(self.h, _p(out), C.c_void_p(dptr), out.nbytes))
        return out

    # ---- profiling (HIP events on the context stream) ----
    def profile(self, enable=True):
        self.check(lib().coeb_profile_enable(self.h, int(enable)))

    def profile_reset(self):
        self.check(lib().coeb_profile_reset(self.h))

    def profile_read(self):
        names = C.create_string_buffer(4096)
        ms = np.zeros(64, np.float64)
        cnt = np.zeros(64, np.int64)
        nk = C.c_int()
        self.check(lib().coeb_profile_read(self.h, names, 4096, _p(ms), _p(cnt), 64, C.byref(nk)))
        nm = names.value.decode().split(",") if nk.value else []
        return {nm[i]: (float(ms[i]), int(cnt[i])) for i in range(nk.value)}


class DeviceBuffer:
    """hipMalloc'ed buffer on the context's device (torch.cuda is not used in-process: the
    torch wheel bundles its own HIP/HSA runtime, which cannot share a process with the
    system ROCm runtime libcoeb_front.so links)."""

    def __init__(self, ctx, nbytes):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        ctx.check(lib().coeb_device_alloc(ctx.h, self.nbytes, C.byref(p)))
        self.ptr = p.value

    def write(self, arr, offset=0):
        arr = np.ascontiguousarray(arr)
        assert offset + arr.nbytes <= self.nbytes
        self.ctx.check(lib().coeb_memcpy_h2d(self.ctx.h, C.c_void_p(self.ptr + offset), _p(arr), arr.nbytes))

    def read(self, dtype=np.uint8, count=None, offset=0):
        dt = np.dtype(dtype)
        count = (self.nbytes - offset) // dt.itemsize if count is None else count
        return self.ctx.download(self.ptr + offset, count * dt.itemsize, dt)

    def free(self):
        if self.ptr is not None and self.ctx.h is not None:
            lib().coeb_device_free(self.ctx.h, C.c_void_p(self.ptr))
        self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class HostBuffer:
    """Page-locked host memory (coeb_host_alloc) viewed as a numpy array: copies between it and
    the device run asynchronously on the DMA engines (coeb_memcpy_*_async)."""

    def __init__(self, nbytes):
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        rc = lib().coeb_host_alloc(self.nbytes, C.byref(p))
        if rc != 0:
            raise CoebError("coeb_host_alloc rc=%d: %s" % (rc, lib().coeb_last_error(None).decode()))
        self.ptr = p.value
        self.array = np.ctypeslib.as_array((C.c_uint8 * self.nbytes).from_address(self.ptr))

    def view(self, dtype, shape=None):
        a = self.array.view(dtype)
        return a if shape is None else a[:int(np.prod(shape))].reshape(shape)

    def free(self):
        if self.ptr is not None:
            self.array = None
            lib().coeb_host_free(C.c_void_p(self.ptr))
        self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def UndistortKeyPoints(ctx, keys, camera, dist):
    """Frame::UndistortKeyPoints (Frame.cc:579-609): mvKeysUn from mvKeys; dist = mDistCoef
    (k1, k2, p1, p2[, k3])."""
    keys = np.ascontiguousarray(keys, KEYPOINT_DTYPE)
    d = np.zeros(5, np.float32)
    d[:len(dist)] = np.asarray(dist, np.float32)
    out = keys.copy()
    ctx.check(lib().coeb_undistort_keypoints(ctx.h, C.byref(camera), _p(d), _p(keys), len(keys), _p(out)))
    return out


def GrabImageRGBD(ctx, imRGB, imD=None, mbRGB=True, mDepthMapFactor=1.0):
    """The input conversions of Tracking::GrabImageRGBD (src/Tracking.cc:212-228) on the device:
    imRGB (H, W) gray, (H, W, 3) RGB/BGR or (H, W, 4) RGBA/BGRA u8 -> gray u8; imD (H, W) uint16
    or float32 -> float32 via convertTo(CV_32F, mDepthMapFactor) (a float32 map with factor 1 is
    kept as is).  mDepthMapFactor is the Tracking member, i.e. 1 / DepthMapFactor of the YAML.
    Returns (gray, depth or None)."""
    img = np.ascontiguousarray(imRGB, np.uint8)
    h, w = img.shape[:2]
    ch = 1 if img.ndim == 2 else img.shape[2]
    gray = np.empty((h, w), np.uint8)
    dep, dtype, dstride = None, 0, 0
    if imD is not None:
        d = np.ascontiguousarray(imD)
        if d.shape != (h, w) or d.dtype not in (np.uint16, np.float32):
            raise ValueError("imD must be (H, W) uint16 or float32")
        dtype = 1 if d.dtype == np.float32 else 0
        dstride = d.strides[0]
        dep = np.empty((h, w), np.float32)
    ctx.check(lib().coeb_rgbd_preprocess(ctx.h, _p(img), ch * w, ch, 1 if mbRGB else 0,
                                         _p(d) if imD is not None else None, dstride, dtype,
                                         C.c_float(mDepthMapFactor), w, h, _p(gray), _p(dep)))
    return gray, dep


def tum_read_file_list(text_or_path):
    """associate.py read_file_list (associate.py:49-69) through coeb_tum_read_list: a dict
    {stamp: [data fields]} of a TUM list file (a path, or the file's text if it holds a newline)."""
    if "\n" not in text_or_path:
        with open(text_or_path) as f:
            text_or_path = f.read()
    raw = text_or_path.encode()
    cap = raw.count(b"\n") + 1
    st = np.zeros(cap, np.float64)
    off = np.zeros(cap, np.int64)
    ln = np.zeros(cap, np.int32)
    n = C.c_int(0)
    rc = lib().coeb_tum_read_list(raw, len(raw), _p(st), _p(off), _p(ln), cap, C.byref(n))
    if rc != 0:
        raise CoebError("coeb_tum_read_list: %d (a stamp field is not a float literal)" % rc)
    sep = re.compile(r"[ ,\t]+")
    return {float(st[i]): [v.strip() for v in sep.split(raw[off[i]:off[i] + ln[i]].decode()) if v.strip()]
            for i in range(n.value)}


def tum_associate(first, second, offset=0.0, max_difference=0.02):
    """associate.py associate (associate.py:71-102) through coeb_tum_associate: the matched
    (stamp_first, stamp_second) pairs ordered by stamp.  first / second: stamp collections (the
    dicts of tum_read_file_list, or arrays)."""
    a = np.ascontiguousarray(list(first), np.float64)
    b = np.ascontiguousarray(list(second), np.float64)
    cap = max(1, min(len(a), len(b)))
    ia = np.zeros(cap, np.int32)
    ib = np.zeros(cap, np.int32)
    n = C.c_int(0)
    rc = lib().coeb_tum_associate(_p(a), len(a), _p(b), len(b), float(offset), float(max_difference), _p(ia), _p(ib),
                                  cap, C.byref(n))
    if rc != 0:
        raise CoebError("coeb_tum_associate: %d" % rc)
    return [(float(a[ia[k]]), float(b[ib[k]])) for k in range(n.value)]


def boxes_from_ros(xyxy):
    """yolov5_ros_msgs/BoundingBoxes (int64 xmin, ymin, xmax, ymax rows) -> float32 [n, 4] as
    ros_rgbd.cc:106-115 builds them."""
    a = np.ascontiguousarray(np.asarray(xyxy, np.int64).reshape(-1, 4))
    out = np.zeros((len(a), 4), np.float32)
    if len(a) and lib().coeb_boxes_from_int64(_p(a), len(a), _p(out)) != 0:
        raise CoebError("coeb_boxes_from_int64 failed")
    return out


class ORBextractor:
    """Drop-in mirror of ORB_SLAM2::ORBextractor (include/ORBextractor.h:44-128)."""

    def __init__(self, nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, device=0, max_width=1280,
                 max_height=960):
        self.ctx = Context(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, device, max_width, max_height, 1)
        t = self.ctx.tables()
        self.nlevels = nlevels
        self.scaleFactor = scaleFactor
        self.mvScaleFactor = list(t.scale[:nlevels])
        self.mvInvScaleFactor = list(t.inv_scale[:nlevels])
        self.mvLevelSigma2 = list(t.sigma2[:nlevels])
        self.mvInvLevelSigma2 = list(t.inv_sigma2[:nlevels])
        self.mnFeaturesPerLevel = list(t.features_per_level[:nlevels])
        self.umax = list(t.umax)

    def __call__(self, image, mask=None, img=None, imD=None, box=None, T_M=None, mask_result=None, blur_flag=None):
        """operator()(image, mask, img, imD, keypoints, descriptors, box, T_M, mask_result, blur_flag).
        mask, img, imD and mask_result are accepted and ignored, as in the reference."""
        image = np.asarray(image)
        if image.size == 0:
            return np.zeros(0, KEYPOINT_DTYPE), None
        assert image.dtype == np.uint8 and image.ndim == 2, "image.type() == CV_8UC1 (ORBextractor.cc:1099)"
        boxes = None if not box else np.asarray(box, np.float32).reshape(-1, 4)
        tm = None if T_M is None or len(T_M) == 0 else np.asarray(T_M, np.float32).reshape(-1, 2)
        bf = None if blur_flag is None or len(blur_flag) == 0 else np.asarray(blur_flag, np.int32)
        return self.ctx.extract(image, boxes, tm, bf)

    def GetLevels(self):
        return self.nlevels

    def GetScaleFactor(self):
        return self.scaleFactor

    def GetScaleFactors(self):
        return list(self.mvScaleFactor)

    def GetInverseScaleFactors(self):
        return list(self.mvInvScaleFactor)

    def GetScaleSigmaSquares(self):
        return list(self.mvLevelSigma2)

    def GetInverseScaleSigmaSquares(self):
        return list(self.mvInvLevelSigma2)


class Frame:
    """The Frame fields SearchByProjection reads (src/Frame.cc / include/Frame.h)."""

    def __init__(self, keys_un, descriptors, u_right=None, Tcw=None, map_points=None, outlier=None):
        self.mvKeysUn = np.ascontiguousarray(keys_un)
        self.N = len(self.mvKeysUn)
        self.mDescriptors = np.ascontiguousarray(descriptors, np.uint8).reshape(self.N, 32) if self.N else \
            np.zeros((0, 32), np.uint8)
        self.mvuRight = np.full(self.N, -1, np.float32) if u_right is None else np.ascontiguousarray(u_right, np.float32)
        self.mTcw = np.eye(4, dtype=np.float32) if Tcw is None else np.ascontiguousarray(Tcw, np.float32)
        # map_points: dict(world_pos [N,3] f32, descriptor [N,32] u8, observations [N] i32, valid [N] u8)
        self.map_points = map_points
        self._outlier = None if outlier is None else np.ascontiguousarray(outlier, np.uint8)
        self.mvpMapPoints = np.full(self.N, -1, np.int32)
        self._mp_obs = None
        self._mp_pos = None

    # the fields below are allocated on first use (a per-frame cost of the Python binding the
    # drop-in latency in bench.py includes; the C++ Tracking thread owns them already)
    @property
    def mvbOutlier(self):
        if self._outlier is None:
            self._outlier = np.zeros(self.N, np.uint8)
        return self._outlier

    @mvbOutlier.setter
    def mvbOutlier(self, v):
        self._outlier = v

    @property
    def mvpMapPointObs(self):
        """Observations() of the MapPoint in mvpMapPoints[i] (-1 = NULL); read by the local-map search."""
        if self._mp_obs is None:
            self._mp_obs = np.full(self.N, -1, np.int32)
        return self._mp_obs

    @mvpMapPointObs.setter
    def mvpMapPointObs(self, v):
        self._mp_obs = v

    @property
    def mvMapPointPos(self):
        """GetWorldPos() of the MapPoint in mvpMapPoints[i]; read by Optimizer.PoseOptimization."""
        if self._mp_pos is None:
            self._mp_pos = np.zeros((self.N, 3), np.float32)
        return self._mp_pos

    @mvMapPointPos.setter
    def mvMapPointPos(self, v):
        self._mp_pos = v


class LocalMap:
    """vpLocalMapPoints after Tracking::SearchLocalPoints ran Frame::isInFrustum on them
    (src/Tracking.cc:1244-1259, src/Frame.cc:445-501): the fields ORBmatcher::SearchByProjection(F, vpMapPoints, th) reads (ORBmatcher.cc:50-80)."""

    def __init__(self, in_view, proj_x, proj_y, proj_xr, level, view_cos, descriptor, observations):
        self.mbTrackInView = np.ascontiguousarray(in_view, np.uint8)
        self.N = len(self.mbTrackInView)
        self.mTrackProjX = np.ascontiguousarray(proj_x, np.float32)
        self.mTrackProjY = np.ascontiguousarray(proj_y, np.float32)
        self.mTrackProjXR = np.ascontiguousarray(proj_xr, np.float32)
        self.mnTrackScaleLevel = np.ascontiguousarray(level, np.int32)
        self.mTrackViewCos = np.ascontiguousarray(view_cos, np.float32)
        self.mDescriptor = np.ascontiguousarray(descriptor, np.uint8).reshape(self.N, 32) if self.N else \
            np.zeros((0, 32), np.uint8)
        self.nObs = np.ascontiguousarray(observations, np.int32)
        for a in (self.mTrackProjX, self.mTrackProjY, self.mTrackProjXR, self.mnTrackScaleLevel, self.mTrackViewCos,
                  self.nObs):
            if len(a) != self.N:
                raise ValueError("LocalMap arrays differ in length")

    def c_struct(self):
        return LocalMapC(self.N, *[C.c_void_p(a.ctypes.data) for a in (
            self.mbTrackInView, self.mTrackProjX, self.mTrackProjY, self.mTrackProjXR, self.mnTrackScaleLevel,
            self.mTrackViewCos, self.mDescriptor, self.nObs)])


class KeyFramePoints:
    """pKF->GetMapPointMatches() snapshot for the relocalisation search (ORBmatcher.cc:1487-1530):
    per slot i, valid (pMP && !isBad()), GetWorldPos(), GetDescriptor(), mfMaxDistance,
    mfMinDistance and pKF->mvKeysUn[i].angle.  sAlreadyFound is passed to SearchByProjection as
    a set of slot indices."""

    def __init__(self, valid, world_pos, descriptor, max_distance, min_distance, angle):
        self.valid = np.ascontiguousarray(valid, np.uint8)
        self.N = len(self.valid)
        self.world_pos = np.ascontiguousarray(world_pos, np.float32).reshape(self.N, 3)
        self.descriptor = np.ascontiguousarray(descriptor, np.uint8).reshape(self.N, 32) if self.N else \
            np.zeros((0, 32), np.uint8)
        self.max_distance = np.ascontiguousarray(max_distance, np.float32)
        self.min_distance = np.ascontiguousarray(min_distance, np.float32)
        self.angle = np.ascontiguousarray(angle, np.float32)
        for a in (self.max_distance, self.min_distance, self.angle):
            if len(a) != self.N:
                raise ValueError("KeyFramePoints arrays differ in length")


class ORBmatcher:
    """Mirror of ORB_SLAM2::ORBmatcher for the tracking projection search."""
    TH_HIGH = 100
    TH_LOW = 50
    HISTO_LENGTH = 30

    def __init__(self, nnratio=0.6, checkOri=True, ctx=None):
        self.mfNNratio = nnratio
        self.mbCheckOrientation = checkOri
        self.ctx = ctx

    @staticmethod
    def DescriptorDistance(a, b):
        a = np.ascontiguousarray(a, np.uint8)
        b = np.ascontiguousarray(b, np.uint8)
        return lib().coeb_descriptor_distance(_p(a), _p(b))

    def SearchByProjection(self, CurrentFrame, second, *args, **kw):
        """The reference's overloads, by the type of the second argument:
          (CurrentFrame, LastFrame: Frame, th, bMono, camera)        ORBmatcher.cc:1329-1471
          (F, vpMapPoints: LocalMap, th=3, camera=...)                 ORBmatcher.cc:44-129
          (F, pKF: KeyFramePoints, sAlreadyFound, th, ORBdist, camera) ORBmatcher.cc:1473-1600"""
        if self.ctx is None:
            self.ctx = Context()
        if isinstance(second, LocalMap):
            return self._search_local_map(CurrentFrame, second, *args, **kw)
        if isinstance(second, KeyFramePoints):
            return self._search_keyframe(CurrentFrame, second, *args, **kw)
        return self._search_last_frame(CurrentFrame, second, *args, **kw)

    def _search_last_frame(self, CurrentFrame, LastFrame, th, bMono, camera):
        mp = LastFrame.map_points
        has = np.ascontiguousarray(mp["valid"], np.uint8)
        outl = np.ascontiguousarray(LastFrame.mvbOutlier, np.uint8)
        xw = np.ascontiguousarray(mp["world_pos"], np.float32)
        desc = np.ascontiguousarray(mp["descriptor"], np.uint8)
        nobs = np.ascontiguousarray(mp["observations"], np.int32)
        keys = np.ascontiguousarray(LastFrame.mvKeysUn)
        lf = LastFrameC(LastFrame.N, has.ctypes.data, outl.ctypes.data, xw.ctypes.data, desc.ctypes.data,
                        nobs.ctypes.data, keys.ctypes.data)
        cf = CurFrameC(CurrentFrame.N, CurrentFrame.mvKeysUn.ctypes.data, CurrentFrame.mDescriptors.ctypes.data,
                       CurrentFrame.mvuRight.ctypes.data)
        # every entry of the result is written by the call (matched index or -1)
        out = np.empty(max(CurrentFrame.N, 1), np.int32)
        nm = C.c_int()
        self.ctx.check(lib().coeb_match_lastframe(self.ctx.h, C.byref(camera), C.byref(cf), C.byref(lf),
                                                  _p(CurrentFrame.mTcw), _p(LastFrame.mTcw), th, int(bMono),
                                                  int(self.mbCheckOrientation), _p(out), C.byref(nm)))
        CurrentFrame.mvpMapPoints = out[:CurrentFrame.N]
        return nm.value


    def _search_keyframe(self, F, kf, sAlreadyFound=(), th=10.0, ORBdist=100, camera=None):
        if camera is None:
            raise ValueError("SearchByProjection(F, pKF, sAlreadyFound, th, ORBdist): camera is required")
        valid = kf.valid.copy()
        for i in sAlreadyFound:
            valid[i] = 0
        cf = CurFrameC(F.N, C.c_void_p(F.mvKeysUn.ctypes.data), C.c_void_p(F.mDescriptors.ctypes.data), None)
        has = np.ascontiguousarray(F.mvpMapPoints >= 0, np.uint8)
        kc = KeyFramePointsC(kf.N, *[C.c_void_p(a.ctypes.data) for a in (
            valid, kf.world_pos, kf.descriptor, kf.max_distance, kf.min_distance, kf.angle)])
        out = np.full(max(F.N, 1), -1, np.int32)
        nm = C.c_int()
        self.ctx.check(lib().coeb_match_keyframe(self.ctx.h, C.byref(camera), C.byref(cf), _p(has), C.byref(kc),
                                                 _p(np.ascontiguousarray(F.mTcw, np.float32)), th, int(ORBdist),
                                                 int(self.mbCheckOrientation), _p(out), C.byref(nm)))
        got = out[:F.N]
        F.mvpMapPoints = np.where(got >= 0, got, F.mvpMapPoints).astype(np.int32)
        return nm.value

    def _search_local_map(self, F, local_map, th=3.0, camera=None):
        if camera is None:
            raise ValueError("SearchByProjection(F, LocalMap, th): camera is required")
        cf = CurFrameC(F.N, C.c_void_p(F.mvKeysUn.ctypes.data), C.c_void_p(F.mDescriptors.ctypes.data),
                       C.c_void_p(F.mvuRight.ctypes.data))
        cobs = np.ascontiguousarray(F.mvpMapPointObs, np.int32)
        lm = local_map.c_struct()
        out = np.full(max(F.N, 1), -1, np.int32)
        nm = C.c_int()
        self.ctx.check(lib().coeb_match_localmap(self.ctx.h, C.byref(camera), C.byref(cf), _p(cobs), C.byref(lm),
                                                 th, self.mfNNratio, _p(out), C.byref(nm)))
        got = out[:F.N]
        hit = got >= 0
        F.mvpMapPoints = np.where(hit, got, F.mvpMapPoints).astype(np.int32)
        if hit.any():
            F.mvpMapPointObs = np.where(hit, local_map.nObs[np.maximum(got, 0)], F.mvpMapPointObs).astype(np.int32)
        return nm.value


class Optimizer:
    """Mirror of ORB_SLAM2::Optimizer for the tracking pose refinement."""

    @staticmethod
    def PoseOptimization(pFrame, camera, ctx):
        F = pFrame
        has = np.ascontiguousarray(F.mvpMapPoints >= 0, np.uint8)
        xw = np.ascontiguousarray(F.mvMapPointPos, np.float32).reshape(F.N, 3) if F.N else np.zeros((1, 3), np.float32)
        fr = PoseFrameC(F.N, C.c_void_p(has.ctypes.data), C.c_void_p(xw.ctypes.data), C.c_void_p(F.mvKeysUn.ctypes.data),
                        C.c_void_p(F.mvuRight.ctypes.data))
        T = np.ascontiguousarray(F.mTcw, np.float32).copy()
        out = np.ascontiguousarray(F.mvbOutlier, np.uint8).copy() if len(F.mvbOutlier) else np.zeros(1, np.uint8)
        nin = C.c_int()
        ctx.check(lib().coeb_pose_optimization(ctx.h, C.byref(camera), C.byref(fr), _p(T), _p(out), C.byref(nin)))
        F.mTcw = T.reshape(4, 4)
        F.mvbOutlier = out[:F.N]
        return nin.value


def make_camera(fx, fy, cx, cy, bf, w, h):
    """Camera + Frame::ComputeImageBounds for an undistorted image (src/Frame.cc:635-641)."""
    return Camera(fx, fy, cx, cy, bf, 0.0, float(w), 0.0, float(h))


# ---- Frame::ProcessMovingObject (src/Frame.cc:311-393) ----
class FlowDebug(C.Structure):
    _fields_ = [("corners_raw", C.c_void_p), ("corners", C.c_void_p), ("ncorners", C.c_void_p),
                ("next_pts", C.c_void_p), ("status", C.c_void_p), ("state", C.c_void_p), ("F", C.c_void_p),
                ("nf", C.c_void_p)]


def _gray(img):
    img = np.ascontiguousarray(img, np.uint8)
    if img.ndim != 2:
        raise ValueError("8UC1 image expected")
    return img, img.shape[1], img.shape[0]


def GoodFeaturesToTrack(ctx, img, max_corners=1000, quality=0.01, min_distance=8.0, k=0.04):
    """cv::goodFeaturesToTrack(img, corners, maxCorners, quality, minDistance, Mat(), 3, true, k)
    as Frame.cc:333 calls it: (n, 2) float32."""
    img, w, h = _gray(img)
    out = np.zeros((max_corners, 2), np.float32)
    n = C.c_int(0)
    ctx.check(lib().coeb_good_features(ctx.h, _p(img), w, h, w, max_corners, quality, min_distance, k, _p(out),
                                       max_corners, C.byref(n)))
    return out[:n.value].copy()


def CornerSubPix(ctx, img, xy, win=10, max_iter=20, eps=0.03):
    """cv::cornerSubPix(img, xy, Size(win, win), Size(-1,-1), TermCriteria(ITER|EPS, max_iter, eps))
    (Frame.cc:334); returns the refined copy."""
    img, w, h = _gray(img)
    xy = np.ascontiguousarray(xy, np.float32).copy()
    ctx.check(lib().coeb_corner_subpix(ctx.h, _p(img), w, h, w, _p(xy), len(xy), win, max_iter, eps))
    return xy


def CalcOpticalFlowPyrLK(ctx, prev, nxt, xy, win=22, max_level=5, max_count=20, eps=0.01):
    """cv::calcOpticalFlowPyrLK(prev, next, xy, next_xy, status, err, Size(win, win), max_level,
    TermCriteria(ITER|EPS, max_count, eps)) (Frame.cc:335): (next_xy, status)."""
    prev, w, h = _gray(prev)
    nxt = np.ascontiguousarray(nxt, np.uint8)
    xy = np.ascontiguousarray(xy, np.float32)
    out = np.zeros_like(xy)
    st = np.zeros(len(xy), np.uint8)
    ctx.check(lib().coeb_optical_flow_pyr_lk(ctx.h, _p(prev), _p(nxt), w, h, w, _p(xy), len(xy), win, max_level,
                                             max_count, eps, _p(out), _p(st)))
    return out, st


def MovingTail(ctx, prev, cur, pxy, nxy, state):
    """SAD check + cv::findFundamentalMat(FM_RANSAC, 0.1, 0.99) + epipolar test (Frame.cc:337-384):
    (T_M or None when F is empty, state after the SAD check, F or None, |F_prepoint|)."""
    prev, w, h = _gray(prev)
    cur = np.ascontiguousarray(cur, np.uint8)
    pxy = np.ascontiguousarray(pxy, np.float32)
    nxy = np.ascontiguousarray(nxy, np.float32)
    st = np.ascontiguousarray(state, np.uint8).copy()
    tm = np.zeros((max(len(pxy), 1), 2), np.float32)
    F = np.zeros(9, np.float64)
    nt, nf = C.c_int(0), C.c_int(0)
    ctx.check(lib().coeb_moving_tail(ctx.h, _p(prev), _p(cur), w, h, w, _p(pxy), _p(nxy), _p(st), len(pxy), _p(tm),
                                     len(tm), C.byref(nt), _p(F), C.byref(nf)))
    if nt.value < 0:
        return None, st, None, nf.value
    return tm[:nt.value].copy(), st, F.reshape(3, 3), nf.value


def ProcessMovingObject(ctx, prev, cur, debug=False):
    """Frame::ProcessMovingObject(imgray, box) with imGrayPre = prev (Frame.cc:311-393): T_M as
    (m, 2) float32, or None when findFundamentalMat returns an empty Mat.  debug=True also
    returns the stage outputs (dict)."""
    prev, w, h = _gray(prev)
    cur = np.ascontiguousarray(cur, np.uint8)
    tm = np.zeros((1024, 2), np.float32)
    nt = C.c_int(0)
    dbg, arrays = None, None
    if debug:
        arrays = dict(corners_raw=np.zeros((1000, 2), np.float32), corners=np.zeros((1000, 2), np.float32),
                      ncorners=np.zeros(1, np.int32), next_pts=np.zeros((1000, 2), np.float32),
                      status=np.zeros(1000, np.uint8), state=np.zeros(1000, np.uint8), F=np.zeros(9, np.float64),
                      nf=np.zeros(1, np.int32))
        dbg = FlowDebug(**{k: _p(v) for k, v in arrays.items()})
    ctx.check(lib().coeb_moving_object_points(ctx.h, _p(prev), _p(cur), w, h, w, _p(tm), len(tm), C.byref(nt),
                                              C.byref(dbg) if dbg is not None else None))
    res = None if nt.value < 0 else tm[:nt.value].copy()
    if not debug:
        return res
    n = int(arrays["ncorners"][0])
    arrays["ncorners"] = n
    arrays["nf"] = int(arrays["nf"][0])
    for k in ("corners_raw", "corners", "next_pts", "status", "state"):
        arrays[k] = arrays[k][:n]
    arrays["F"] = arrays["F"].reshape(3, 3)
    return res, arrays
