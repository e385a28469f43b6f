"""Device-resident batch pipeline: extract F frames and match each to its predecessor.

The per-frame front end of Tracking::GrabImageRGBD -> Frame(RGB-D) -> ExtractORB and
Tracking::TrackWithMotionModel -> SearchByProjection (src/Tracking.cc:207-233, 933-958),
for a batch of frames already resident in HBM.  Frame 0 of a batch is the halo: it is
extracted so frame 1 can be matched, and is not counted as a processed frame.
"""
import numpy as np

from . import Context, KEYPOINT_DTYPE, make_camera, synth


class BatchPipeline:
    def __init__(self, width, height, nframes, nfeatures=1000, scale_factor=1.2, nlevels=8, device=0,
                 camera=None):
        self.W, self.H, self.F = width, height, nframes
        self.ctx = Context(nfeatures, scale_factor, nlevels, 20, 7, device, width, height, nframes)
        self.cam = camera or make_camera(synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF,
                                         width, height)
        self.gray = None
        self.depth = None
        self.dTcw = None
        self.Tcw = np.stack([np.eye(4, dtype=np.float32)] * nframes)
        self.dyn = None
        self.host_frames = None

    def load(self, frames, depth=None, Tcw=None, dyn=None):
        """frames: (F, H, W) uint8; depth: (F, H, W) float32; Tcw: (F, 4, 4) pose of frame f
        relative to frame f-1; dyn: per-frame (boxes, T_M, blur_flag) or None."""
        frames = np.ascontiguousarray(frames, np.uint8)
        assert frames.shape == (self.F, self.H, self.W)
        self.gray = self.ctx.upload(frames)
        self.host_frames = frames
        if depth is None:
            depth = np.broadcast_to(synth.make_depth(self.W, self.H), (self.F, self.H, self.W))
        self.depth = self.ctx.upload(np.ascontiguousarray(depth, np.float32))
        if Tcw is not None:
            self.Tcw = np.ascontiguousarray(Tcw, np.float32)
        self.dTcw = self.ctx.upload(self.Tcw.reshape(self.F, 16))     # poses resident like the frames
        if dyn is not None:
            boxes, tms, blurs = [], [], []
            box_off, tm_off = [0], [0]
            for b, t, bl in dyn:
                b = np.zeros((0, 4), np.float32) if b is None else np.asarray(b, np.float32).reshape(-1, 4)
                t = np.zeros((0, 2), np.float32) if t is None else np.asarray(t, np.float32).reshape(-1, 2)
                bl = np.zeros(len(b), np.int32) if bl is None else np.asarray(bl, np.int32)
                blf = np.zeros(len(b), np.int32)
                blf[:min(len(bl), len(b))] = bl[:len(b)]
                boxes.append(b)
                tms.append(t)
                blurs.append(blf)
                box_off.append(box_off[-1] + len(b))
                tm_off.append(tm_off[-1] + len(t))
            self.dyn = (np.concatenate(boxes), np.asarray(box_off, np.int32), np.concatenate(tms),
                        np.asarray(tm_off, np.int32), np.concatenate(blurs))
        self.ctx.synchronize()

    def run(self, match=True, th=15.0, nobs=2, pose=False):
        """Enqueue one step (extraction of F frames + F-1 matches, and with pose=True the
        motion-model PoseOptimization of every matched frame); does not synchronise."""
        if self.dyn is not None:
            b, bo, t, to, bl = self.dyn
            self.ctx.extract_batch_device(self.gray.ptr, self.F, self.W, self.H, b, bo, t, to, bl)
        else:
            self.ctx.extract_batch_device(self.gray.ptr, self.F, self.W, self.H)
        if match:
            self.ctx.match_batch_device_tcw(self.depth.ptr, self.F, self.W, self.H, self.cam, self.dTcw.ptr, th, nobs)
            if pose:
                self.ctx.pose_batch_device(self.cam, self.F, self.dTcw.ptr)

    def synchronize(self):
        self.ctx.synchronize()

    def run_host(self, frames, staging=None):
        """One step with host buffers at both ends (the PCIe-inclusive rate):
        upload `frames` (F, H, W) u8, extract + match, copy keypoints, descriptors, counts and
        match indices back.  Copies are synchronous on the context stream (not overlapped).
        Returns the staging dict of host arrays (reused across calls)."""
        kp_ptr, desc_ptr, cnt_ptr, kcap = self.ctx.batch_results()
        if staging is None:
            staging = dict(kps=np.empty(28 * kcap * self.F, np.uint8), desc=np.empty(32 * kcap * self.F, np.uint8),
                           counts=np.empty(self.F, np.int32), match=np.empty(kcap * self.F, np.int32),
                           nmatch=np.empty(self.F, np.int32))
        self.gray.write(frames)
        self.run()
        kp_ptr, desc_ptr, cnt_ptr, kcap = self.ctx.batch_results()
        m_ptr, n_ptr = self.ctx.batch_match_results()
        self.ctx.download_into(cnt_ptr, staging["counts"])
        self.ctx.download_into(kp_ptr, staging["kps"])
        self.ctx.download_into(desc_ptr, staging["desc"])
        self.ctx.download_into(m_ptr, staging["match"])
        self.ctx.download_into(n_ptr, staging["nmatch"])
        return staging

    def results(self):
        """Host copies: list of (keypoints, descriptors) per frame, match arrays, nmatches."""
        kp_ptr, desc_ptr, cnt_ptr, kcap = self.ctx.batch_results()
        counts = self.ctx.download(cnt_ptr, 4 * self.F, np.int32)
        kps = self.ctx.download(kp_ptr, 28 * kcap * self.F, np.uint8).view(KEYPOINT_DTYPE).reshape(self.F, kcap)
        desc = self.ctx.download(desc_ptr, 32 * kcap * self.F, np.uint8).reshape(self.F, kcap, 32)
        out = [(kps[f, :counts[f]].copy(), desc[f, :counts[f]].copy()) for f in range(self.F)]
        m_ptr, n_ptr = self.ctx.batch_match_results()
        matches, nm = None, None
        if m_ptr and n_ptr and self.F > 1:
            nm = self.ctx.download(n_ptr, 4 * self.F, np.int32)
            mm = self.ctx.download(m_ptr, 4 * kcap * self.F, np.int32).reshape(self.F, kcap)
            matches = [None] + [mm[f, :counts[f]].copy() for f in range(1, self.F)]
            nm = [None] + [int(x) for x in nm[1:]]
        return out, matches, nm

    def pose_results(self):
        """Host copies after run(pose=True): Tcw (F, 4, 4) (frame 0 unused), inliers per frame
        (0: not tracked), outlier flags per frame (frame 0: None)."""
        kp_ptr, _, cnt_ptr, kcap = self.ctx.batch_results()
        counts = self.ctx.download(cnt_ptr, 4 * self.F, np.int32)
        t_ptr, n_ptr, o_ptr = self.ctx.batch_pose_results()
        T = self.ctx.download(t_ptr, 64 * self.F, np.float32).reshape(self.F, 4, 4)
        nin = self.ctx.download(n_ptr, 4 * self.F, np.int32)
        outl = self.ctx.download(o_ptr, kcap * self.F, np.uint8).reshape(self.F, kcap)
        return T, [int(x) for x in nin], [None] + [outl[f, :counts[f]].copy() for f in range(1, self.F)]

    def close(self):
        for b in (self.gray, self.depth, self.dTcw):
            if b is not None:
                b.free()
        self.ctx.close()
