"""Device-resident batch pipeline: extract F frames and match each to its predecessor.

The per-frame front end of Tracking::GrabImageRGBD -> Frame(RGB-D) -> ExtractORB and
Tracking::TrackWithMotionModel -> SearchByProjection (src/Tracking.cc:207-233, 933-958),
for a batch of frames already resident in HBM.  Frame 0 of a batch is the halo: it is
extracted so frame 1 can be matched, and is not counted as a processed frame.
"""
import numpy as np

import ctypes as C

from . import Context, DeviceBuffer, HostBuffer, KEYPOINT_DTYPE, lib, make_camera, synth


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
        self.frame_boxes = None      # (boxes, box_off) for run(frame=True)
        self.raw = None              # (image, channels, rgb_order, depth, depth_type, factor) for run(rgbd=True)

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

    def load_rgbd(self, images, depth, depth_factor, rgb_order=1, Tcw=None):
        """Raw GrabImageRGBD input resident on the device: images (F, H, W[, C]) u8 with C = 1, 3
        or 4, depth (F, H, W) u16 or f32, mDepthMapFactor = depth_factor (1 / DepthMapFactor);
        run(rgbd=True) converts them into the batch's gray frames and float depth first."""
        images = np.ascontiguousarray(images, np.uint8)
        ch = 1 if images.ndim == 3 else images.shape[3]
        assert images.shape[:3] == (self.F, self.H, self.W)
        depth = np.ascontiguousarray(depth)
        assert depth.shape == (self.F, self.H, self.W) and depth.dtype in (np.uint16, np.float32)
        from . import DEPTH_U16, DEPTH_F32
        for b in (self.raw[0], self.raw[3]) if self.raw else ():
            b.free()
        self.raw = (self.ctx.upload(images), ch, rgb_order, self.ctx.upload(depth),
                    DEPTH_U16 if depth.dtype == np.uint16 else DEPTH_F32, float(np.float32(depth_factor)))
        if self.gray is None:
            self.gray = self.ctx.alloc(self.F * self.H * self.W)
            self.depth = self.ctx.alloc(4 * self.F * self.H * self.W)
        if Tcw is not None:
            self.Tcw = np.ascontiguousarray(Tcw, np.float32)
        if self.dTcw is None or Tcw is not None:
            self.dTcw = self.ctx.upload(self.Tcw.reshape(self.F, 16))
        self.ctx.synchronize()

    def run(self, match=True, th=15.0, nobs=2, pose=False, frame=False, track=False, nkf=2, rgbd=False):
        """Enqueue one step (extraction of F frames + F-1 matches, and with pose=True the
        motion-model PoseOptimization of every matched frame, with track=True also TrackLocalMap:
        local map of KeyFrames f-1, f-2 -> SearchByProjection -> PoseOptimization, BASELINE
        configs[4]); does not synchronise.  frame=True
        runs the whole RGB-D Frame constructor instead of the extraction alone: T_M from the
        previous frame (ProcessMovingObject), blur flags of the boxes set by set_frame_boxes(),
        masked extraction (coeb_frame_batch_device)."""
        if rgbd:
            img, ch, order, dep, dt, fac = self.raw
            self.ctx.rgbd_preprocess_batch_device(img.ptr, ch, order, dep.ptr, dt, fac, self.F, self.W, self.H,
                                                  self.gray.ptr, self.depth.ptr)
        if frame:
            b, o = self.frame_boxes if self.frame_boxes is not None else (None, None)
            self.ctx.frame_batch_device(self.gray.ptr, self.F, self.W, self.H, b, o)
        elif self.dyn is not None:
            b, bo, t, to, bl = self.dyn
            self.ctx.extract_batch_device(self.gray.ptr, self.F, self.W, self.H, b, bo, t, to, bl)
        else:
            self.ctx.extract_batch_device(self.gray.ptr, self.F, self.W, self.H)
        if match:
            self.ctx.match_batch_device_tcw(self.depth.ptr, self.F, self.W, self.H, self.cam, self.dTcw.ptr, th, nobs)
            if pose or track:
                self.ctx.pose_batch_device(self.cam, self.F, self.dTcw.ptr)
            if track:
                self.ctx.track_local_map_batch_device(self.cam, self.F, nkf)

    def set_frame_boxes(self, boxes_per_frame):
        """YOLO boxes of every frame (list of (n_f, 4) xyxy) for run(frame=True)."""
        bl = [np.zeros((0, 4), np.float32) if b is None else np.asarray(b, np.float32).reshape(-1, 4)
              for b in boxes_per_frame]
        off = np.zeros(len(bl) + 1, np.int32)
        off[1:] = np.cumsum([len(b) for b in bl])
        self.frame_boxes = (np.concatenate(bl) if off[-1] else np.zeros((0, 4), np.float32), off)

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

    def frame(self, f, track=False):
        """Host copies of frame f's results alone (a few KB instead of the whole batch): its
        keypoints and descriptors, and for f >= 1 its SearchByProjection count and match indices;
        with track=True also the configs[4] loop's per-frame records as track_results() gives
        them (motion-model pose T1 / inliers nin1, TrackLocalMap pose T / inliers, nmatchesMap,
        local-map matches, outlier flags, state)."""
        if not 0 <= f < self.F:
            raise IndexError("frame %d outside the batch of %d" % (f, self.F))
        c = self.ctx
        kp_ptr, desc_ptr, cnt_ptr, kcap = c.batch_results()
        n = int(c.download(cnt_ptr + 4 * f, 4, np.int32)[0])
        out = dict(kps=c.download(kp_ptr + 28 * kcap * f, 28 * n).view(KEYPOINT_DTYPE),
                   desc=c.download(desc_ptr + 32 * kcap * f, 32 * n).reshape(n, 32))
        if f == 0:
            return out
        m_ptr, n_ptr = c.batch_match_results()
        out["nmatch"] = int(c.download(n_ptr + 4 * f, 4, np.int32)[0])
        out["match"] = c.download(m_ptr + 4 * kcap * f, 4 * n, np.int32)
        if not track:
            return out
        t_ptr, ni_ptr, _ = c.batch_pose_results()
        out["T1"] = c.download(t_ptr + 64 * f, 64, np.float32).reshape(4, 4)
        out["nin1"] = int(c.download(ni_ptr + 4 * f, 4, np.int32)[0])
        t_ptr, ni_ptr, nm_ptr, nl_ptr, lm_ptr, o_ptr = c.batch_track_results()
        out["T"] = c.download(t_ptr + 64 * f, 64, np.float32).reshape(4, 4)
        out["ninliers"] = int(c.download(ni_ptr + 4 * f, 4, np.int32)[0])
        out["nmatches_map"] = int(c.download(nm_ptr + 4 * f, 4, np.int32)[0])
        out["nlocal"] = int(c.download(nl_ptr + 4 * f, 4, np.int32)[0])
        out["local_match"] = c.download(lm_ptr + 4 * kcap * f, 4 * n, np.int32)
        out["outlier"] = c.download(o_ptr + kcap * f, n, np.uint8)
        if out["nmatch"] < 20 or out["nmatches_map"] < 10:           # the rule of track_results()
            out["state"] = 0
        else:
            out["state"] = 2 if out["ninliers"] >= 30 else 1
        return out

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

    def track_results(self):
        """Host copies after run(track=True), per frame (index 0 = halo, unused): Tcw (F, 4, 4)
        after TrackLocalMap, second-PoseOptimization inliers, nmatchesMap, local-map matches
        (count and per-keypoint local index), outlier flags, and the tracking state (0: the
        motion model failed, 1: TrackLocalMap failed (< 30 inliers, Tracking.cc:1040-1046),
        2: tracked)."""
        _, _, cnt_ptr, kcap = self.ctx.batch_results()
        counts = self.ctx.download(cnt_ptr, 4 * self.F, np.int32)
        t_ptr, n_ptr, m_ptr, nl_ptr, lm_ptr, o_ptr = self.ctx.batch_track_results()
        T = self.ctx.download(t_ptr, 64 * self.F, np.float32).reshape(self.F, 4, 4)
        nin = self.ctx.download(n_ptr, 4 * self.F, np.int32)
        nmap = self.ctx.download(m_ptr, 4 * self.F, np.int32)
        nloc = self.ctx.download(nl_ptr, 4 * self.F, np.int32)
        lm = self.ctx.download(lm_ptr, 4 * kcap * self.F, np.int32).reshape(self.F, kcap)
        outl = self.ctx.download(o_ptr, kcap * self.F, np.uint8).reshape(self.F, kcap)
        _, _, nms = self.results()
        state = [None]
        for f in range(1, self.F):
            if nms[f] < 20 or nmap[f] < 10:
                state.append(0)
            else:
                state.append(2 if nin[f] >= 30 else 1)
        return dict(T=T, ninliers=[int(x) for x in nin], nmatches_map=[int(x) for x in nmap],
                    nlocal=[int(x) for x in nloc], local_match=[None] + [lm[f, :counts[f]].copy() for f in range(1, self.F)],
                    outlier=[None] + [outl[f, :counts[f]].copy() for f in range(1, self.F)], state=state, stride=kcap)

    def close(self):
        for b in (self.gray, self.depth, self.dTcw) + ((self.raw[0], self.raw[3]) if self.raw else ()):
            if b is not None:
                b.free()
        self.ctx.close()


class HostStream:
    """Host buffers in, host buffers out, with copy / kernel overlap (the PCIe-inclusive rate,
    DESIGN.md s6).

    mode="ring" (default): one context computes the batches in order; an upload queue
    (coeb_copyq) fills a ring of three device input buffers.  Batch i: the queue waits for the
    marker "kernels of batch i - 3 done" (its buffer is free), uploads, records "upload i done";
    the context waits for that marker, runs the kernels on buffer i % 3, records "kernels i
    done", downloads keypoints / descriptors / counts / matches into output set i % 2 on its own
    stream and records "results i in host memory" (what wait(i) waits for).  The upload queue
    never waits for the batch just before it, so uploads run back to back at the link rate
    beside the kernels and downloads (79 MB per 257 frames at ~57 GB/s = 1.38 ms; kernels 1.07 ms
    + download 0.31 ms on the context stream): one upload per batch in steady state.

    The two-context forms, kept for comparison (profiles/r02/v3/hoststream_modes.txt):

    mode="slot": batch i (slot k = i % 2) is, in order on slot k's own stream, the
    upload of its gray frames from page-locked host memory, its kernels, and the download of
    keypoints / descriptors / counts / matches into slot k's page-locked output buffers.  Batch
    i's upload also waits for batch i - 1's upload (one event through an idle "gate" queue): left
    free, the two slots fall into phase (both upload at half rate, both compute at once) and a
    batch took 2.7 ms.  Staggered, batch i + 1 uploads while batch i computes and downloads.
    Uploads are the bound (79 MB per 257 frames at ~57 GB/s = 1.38 ms vs 1.07 ms of kernels +
    0.31 ms of download), and a slot's next upload starts as its own download ends: one upload
    per batch in steady state.

    mode="copyq": one copy queue (coeb_copyq) carries every upload and download, ordered against
    the slots by device-side events (shared_queue=False gives each slot a download queue of its
    own): the upload of batch i + 1 queued behind batch i - 1's download, which waits for its
    kernels (profiles/r02/v3/hoststream_copyq_timeline.txt).

    Either way submit() never blocks the host.  Results of batch i are readable after wait(i) and
    stay so until batch i + 2 is submitted (its download reuses slot i % 2's host buffers).  The
    ring mode needs three streams (context, copy queue, downloads), which HIP's default of 4
    hardware queues per process gives each a queue of their own; the slot modes' two contexts
    need more (GPU_MAX_HW_QUEUES = 16), else their streams share queues and the overlap
    disappears."""

    def __init__(self, width, height, nframes, nfeatures=1000, device=0, depth=None, Tcw=None, shared_queue=True,
                 mode="ring"):
        if mode not in ("ring", "slot", "copyq"):
            raise ValueError("HostStream mode must be 'ring', 'slot' or 'copyq'")
        self.mode = mode
        self.W, self.H, self.F = width, height, nframes
        nslots = 1 if mode == "ring" else 2
        self.slots = [BatchPipeline(width, height, nframes, nfeatures=nfeatures, device=device) for _ in range(nslots)]
        zero = np.zeros((nframes, height, width), np.uint8)
        for sl in self.slots:
            sl.load(zero, depth=depth, Tcw=Tcw)
            sl.run()                                   # sizes every device buffer once
            sl.synchronize()
        kp_ptr, desc_ptr, cnt_ptr, kcap = self.slots[0].ctx.batch_results()
        self.kcap = kcap
        F = nframes
        self.sizes = dict(kps=28 * kcap * F, desc=32 * kcap * F, counts=4 * F, match=4 * kcap * F, nmatch=4 * F)
        self.out = [{k: HostBuffer(n) for k, n in self.sizes.items()} for _ in range(2)]
        self.inflight = []
        self.pending_dl = None              # batch whose download is not enqueued yet (copyq mode)
        self.up, self.down = None, []
        self.markers, self.ring = [], []
        L = lib()
        if mode == "ring":
            sl = self.slots[0]
            nb = nframes * height * width
            self.ring = [sl.gray] + [DeviceBuffer(sl.ctx, nb) for _ in range(self.NRING - 1)]
            self.up = L.coeb_copyq_create(sl.ctx.h)
            self.markers = [[L.coeb_marker_create(sl.ctx.h) for _ in range(self.NMARK)] for _ in range(3)]
            if not self.up or not all(all(m) for m in self.markers):
                raise RuntimeError("HostStream: copy queue / marker creation failed: %s" %
                                   L.coeb_last_error(None).decode())
            self.updone, self.kdone, self.dldone = self.markers
            return
        if mode == "slot":
            # gate: an otherwise idle copy queue that only carries event waits, so slot k's
            # upload can wait for the other slot's upload (and nothing after it) to finish
            self.gate = L.coeb_copyq_create(self.slots[0].ctx.h)
            if not self.gate:
                raise RuntimeError("coeb_copyq_create failed: %s" % L.coeb_last_error(None).decode())
            self.down = [self.gate]
            return
        self.up = L.coeb_copyq_create(self.slots[0].ctx.h)
        self.down = [self.up, self.up] if shared_queue else [L.coeb_copyq_create(sl.ctx.h) for sl in self.slots]
        if not self.up or not all(self.down):
            raise RuntimeError("coeb_copyq_create failed: %s" % L.coeb_last_error(None).decode())

    def _chk(self, rc):
        if rc != 0:
            raise RuntimeError("coeb rc=%d: %s" % (rc, lib().coeb_last_error(None).decode()))

    def _downloads(self, k, slot=None):
        """(host, device, bytes) of the result copies into output set k from slot `slot` (k)."""
        c = self.slots[k if slot is None else slot].ctx
        kp_ptr, desc_ptr, cnt_ptr, _ = c.batch_results()
        m_ptr, n_ptr = c.batch_match_results()
        o = self.out[k]
        return [(o[name].ptr, dptr, self.sizes[name]) for name, dptr in
                (("counts", cnt_ptr), ("kps", kp_ptr), ("desc", desc_ptr), ("match", m_ptr), ("nmatch", n_ptr))]

    NRING = 3          # device input buffers of the ring mode
    NMARK = 8          # markers per kind (a marker is re-recorded NMARK batches later)

    def submit(self, i, host_frames):
        """Enqueue batch i (host_frames: a HostBuffer of F*H*W gray bytes); returns at once (the
        device orders it after the batches before it)."""
        L = lib()
        nb = self.F * self.H * self.W
        if self.mode == "ring":
            sl, c = self.slots[0], self.slots[0].ctx
            buf, r = self.ring[i % self.NRING], i % self.NMARK
            if i >= self.NRING:        # the kernels that read this input buffer last are done
                self._chk(L.coeb_copyq_wait_marker(self.up, self.kdone[(i - self.NRING) % self.NMARK]))
            self._chk(L.coeb_copyq_h2d(self.up, C.c_void_p(buf.ptr), C.c_void_p(host_frames.ptr), nb))
            self._chk(L.coeb_marker_record_copyq(self.updone[r], self.up))
            self._chk(L.coeb_ctx_wait_marker(c.h, self.updone[r]))
            sl.gray = buf
            sl.run()
            self._chk(L.coeb_marker_record_ctx(self.kdone[r], c.h))
            for hptr, dptr, n in self._downloads(i % 2, 0):
                self._chk(L.coeb_memcpy_d2h_async(c.h, C.c_void_p(hptr), C.c_void_p(dptr), n))
            self._chk(L.coeb_marker_record_ctx(self.dldone[r], c.h))
            self.inflight.append(i)
            return
        k = i % 2
        sl, c = self.slots[k], self.slots[k].ctx
        if self.mode == "slot":
            # uploads one after another (each at the full link rate) instead of two at once: the
            # slots then stay half a period apart and batch i + 1 uploads while batch i computes
            self._chk(L.coeb_ctx_after_copyq(c.h, self.gate))
            self._chk(L.coeb_memcpy_h2d_async(c.h, C.c_void_p(sl.gray.ptr), C.c_void_p(host_frames.ptr), nb))
            self._chk(L.coeb_copyq_after_ctx(self.gate, c.h))
            sl.run()
            for hptr, dptr, n in self._downloads(k):
                self._chk(L.coeb_memcpy_d2h_async(c.h, C.c_void_p(hptr), C.c_void_p(dptr), n))
            self.inflight.append(i)
            return
        # copyq: batch i's upload is queued before batch i - 1's download, so on a shared copy
        # queue the upload does not wait behind batch i - 1's kernels
        self._chk(L.coeb_copyq_after_ctx(self.up, c.h))
        self._chk(L.coeb_copyq_h2d(self.up, C.c_void_p(sl.gray.ptr), C.c_void_p(host_frames.ptr), nb))
        self._chk(L.coeb_ctx_after_copyq(c.h, self.up))
        if self.down[k] != self.up:
            self._chk(L.coeb_ctx_after_copyq(c.h, self.down[k]))
        sl.run()
        self._flush_download()
        self.pending_dl = i
        self.inflight.append(i)

    def _flush_download(self):
        i = self.pending_dl
        if i is None:
            return
        self.pending_dl = None
        k = i % 2
        L = lib()
        self._chk(L.coeb_copyq_after_ctx(self.down[k], self.slots[k].ctx.h))
        for hptr, dptr, n in self._downloads(k):
            self._chk(L.coeb_copyq_d2h(self.down[k], C.c_void_p(hptr), C.c_void_p(dptr), n))

    def wait(self, i):
        """Block until batch i's results are in its slot's host buffers (with later batches of
        the same slot submitted, this also waits for them)."""
        if self.mode == "copyq" and self.pending_dl is not None and self.pending_dl <= i:
            self._flush_download()
        if i in self.inflight:
            if self.mode == "ring":
                self._chk(lib().coeb_marker_synchronize(self.dldone[i % self.NMARK]))
            elif self.mode == "slot":
                self.slots[i % 2].synchronize()
            else:
                self._chk(lib().coeb_copyq_synchronize(self.down[i % 2]))
            self.inflight = [j for j in self.inflight if j % 2 != i % 2 or j > i]
        return self.out[i % 2]

    def results(self, i):
        """Per-frame (keypoints, descriptors), matches and nmatches of batch i (after wait(i))."""
        o = self.out[i % 2]
        counts = o["counts"].view(np.int32)
        kps = o["kps"].view(np.uint8).view(KEYPOINT_DTYPE).reshape(self.F, self.kcap)
        desc = o["desc"].view(np.uint8).reshape(self.F, self.kcap, 32)
        mm = o["match"].view(np.int32).reshape(self.F, self.kcap)
        nm = o["nmatch"].view(np.int32)
        out = [(kps[f, :counts[f]].copy(), desc[f, :counts[f]].copy()) for f in range(self.F)]
        return out, [None] + [mm[f, :counts[f]].copy() for f in range(1, self.F)], [None] + [int(x) for x in nm[1:]]

    def close(self):
        L = lib()
        for q in set([self.up] + self.down):
            if q:
                L.coeb_copyq_destroy(q)
        self.up, self.down = None, []
        for sl in self.slots:
            sl.synchronize()
        for kind in self.markers:
            for m in kind:
                if m:
                    L.coeb_marker_destroy(m)
        self.markers = []
        for b in self.ring[1:]:
            b.free()
        if self.ring:
            self.slots[0].gray = self.ring[0]
        self.ring = []
        for sl in self.slots:
            sl.close()
        for o in self.out:
            for b in o.values():
                b.free()
