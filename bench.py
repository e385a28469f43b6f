#!/usr/bin/env python3
"""Benchmark: frames/s of the ORB front end (extract + Hamming match to the previous frame)
on synthetic 640x480 input, 8 levels, 1000 keypoints (BASELINE.json configs[1]).

A step = one pass of the hot path over one batch of B frames already resident in HBM:
extraction of B+1 frames (frame 0 is the halo that gives frame 1 its LastFrame) and B
SearchByProjection calls (th = 15, retried at 30 below 20 matches, Tracking.cc:947-958).
Only the B matched frames are counted.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): one
process per GPU, each with its own batch (frames are independent; no data-path collective,
scaling "weak").  torch.distributed (gloo) is used only for the barrier and the max-over-
ranks of the timed interval; the GPU work is libcoeb_front.so's (torch.cuda is never
initialised: the torch wheel bundles its own HIP runtime).
"""
import argparse
import json
import math
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "coeb-slam_amd"))
# Hardware queues per process: the bench takes the environment's GPU_MAX_HW_QUEUES (the GPU box
# exports 4, HIP's default) and records it in the line (config.hw_queues).  Measured on this build:
# with 4 queues the pipelines' side streams share one queue, and that is the fastest setting
# (8 or 16 queues: 1-2 % slower; DESIGN.md s0, profiles/r05/s1).
HW_QUEUES = os.environ.get("GPU_MAX_HW_QUEUES")

import numpy as np  # noqa: E402

METRIC = "frames/sec ORB extract+match @640x480/1000 kp; 1/2/4/8 GPU + %HBM roofline"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md)
CONFIGS = {
    # batch = matched frames per step per GPU, split over `pipelines` contexts whose kernels overlap.
    # A and C: 2048 as 2 x 1024.  One pipeline measured 208 / 250 / 257 / 269 / 265 k frames/s at
    # 128 / 256 / 512 / 1024 / 2048 frames (profiles/r02/v3/batch_sweep.txt: 1024 frames give every
    # launch >= 4 workgroups per CU, including the small pyramid levels and the matcher); two 1024-frame
    # pipelines 275 k (profiles/r02/v4/pipelines_ab.txt).  Round 5 (profiles/r05/sched): with the side
    # stream, pipelines x frames 1 x 2048 356.8 k, 2 x 1024 361.4 k, 3 x 683 365.5 k, 3 x 1024 368.0 k,
    # 4 x 512 356.1 k, 4 x 1024 363.5 k frames/s; without it 2 x 1024 347-350 k.  D: 1024 as 2 x 512 -- its flow kernels
    # (cornerSubPix, LK, findFundamentalMat, PoseOptimization) are latency bound, one workgroup or wave
    # per corner / pair / frame, so they need many frames in flight: batch x pipelines 256 x 1 measured
    # 51.4 k frames/s, 256 x 2 57.0 k, 512 x 2 61.6 k, 1024 x 2 64.5 k, 2048 x 2 64.5 k, 2048 x 4 58.1 k
    # (profiles/r03/s4/benchD_batch.txt).
    # A: each pipeline's side stream created with its context (COEB_SIDE_EAGER=1), so the six streams
    # take the box's 4 hardware queues in (context, side) pairs: 8.27-8.31 ms per step against
    # 8.33-8.38 when they are created at the first extraction (profiles/r05/s38, s38b; C and D: no gain)
    "A": dict(w=640, h=480, nfeatures=1000, batch=3072, pipelines=3, side_eager=True,
              workload="640x480, 8-level pyramid, 1000 kp, extract + Hamming match to prev frame (BASELINE configs[1])"),
    # B: the fixed 512-frame batch of BASELINE configs[3] as 2 pipelines per GPU (per-rank shards of
    # 64-256 frames ran 5-10 % faster with 2 than with 1, profiles/r03/s5/shardB_pipelines.txt)
    "B": dict(w=1280, h=960, nfeatures=2000, pipelines=2, workload="1280x960, 8-level pyramid, 2000 kp, extract + match (BASELINE configs[3] shape)"),
    # C: the three pipelines share one extraction side stream (3 context streams + 1 side stream on the
    # box's 4 hardware queues): 8.65-8.89 ms per step against 9.01-9.15 with a side stream each; for A
    # and D the shared stream measured slower (8.51-8.54 vs 8.27-8.36 ms, 13.63-13.76 vs 13.15-13.21,
    # profiles/r05/s19, s20)
    "C": dict(w=640, h=480, nfeatures=1000, dyn=True, batch=3072, pipelines=3, side_stream="shared",
              workload="640x480, 1000 kp, YOLO-bbox dynamic mask (2 boxes, 60 T_M points, blur_flag [0,1]) + "
                       "depth association (ComputeStereoFromRGBD) + match to prev frame (BASELINE configs[2])"),
    # D: two pipelines (three or four: 68.7-73.9 k); per-GPU batch 1024 / 1536 / 2048 / 3072 frames:
    # 81.9-82.6 / 82.6-83.4 / 83.0-83.8 / 83.9-84.4 k frames/s (profiles/r05/s31, s31b): 3072 as for A and C
    "D": dict(w=640, h=480, nfeatures=1000, chain=True, batch=3072, pipelines=2,
              workload="640x480, 1000 kp, the full Tracking::GrabImageRGBD loop per frame (BASELINE configs[4]): "
                       "RGB + 16U depth conversion, Frame ctor (ProcessMovingObject T_M from the previous frame, "
                       "YOLO-box blur flags, dynamic mask, ORB extraction), TrackWithMotionModel (SearchByProjection "
                       "th 15 + retry, PoseOptimization, outlier discard), TrackLocalMap (local map of KeyFrames f-1 "
                       "and f-2 through isInFrustum, SearchByProjection th 3, PoseOptimization)",
              data="synthetic tracking sequence (TUM-like rectangles + noise, (+2,+1) px/frame camera motion, a "
                   "bouncing 120x160 textured object with its YOLO box; RGB = gray x 3, 16U depth 10000 = 2 m)"),
}
# COEB_BENCH_ONE_DEVICE=1 rehearses --gpus N (threads, shards, barriers, max over ranks) with every
# rank on device 0 of a one-GPU box; its lines carry "rehearsal_one_device" and measure nothing.
ONE_DEVICE = os.environ.get("COEB_BENCH_ONE_DEVICE") == "1"
DEPTH_MAP_FACTOR = 1.0 / 5000.0     # mDepthMapFactor = 1 / DepthMapFactor (TUM yaml: 5000)
CPU_CAVEAT = ("the oracle is a scalar C restatement of ORBextractor/ORBmatcher with the OpenCV primitives "
              "(FAST, resize, GaussianBlur, LK, ...) restated without SIMD: real OpenCV 3.4 vectorises them, so the "
              "reference binary runs faster than this port (SURVEY.md s8(d)); the reference itself is unbuildable here "
              "(no OpenCV/g2o/DBoW2 in the image)")

CHAIN_WARMUP = 20    # 20 warm-up frames before the timed ones


# kernels that read the frames' pixels (the s8(d) image-byte rule applies to them)
IMAGE_KERNELS = ("k_fast", "k_describe", "k_blur", "k_blur_rows", "k_pyr_level", "k_pyr_rows", "k_rgbd_batch",
                 "k_gf_response", "k_subpix", "k_lk", "k_pyr_down", "k_sharr")


def step_kwargs(cfg):
    """BatchPipeline.run() arguments of one step of `cfg`."""
    if cfg.get("chain"):
        return dict(rgbd=True, frame=True, track=True)
    return dict(pose=bool(cfg.get("pose")))


def load_batch(bp, cfg, w, h, F, first):
    """Synthetic input of `cfg` for global frames first .. first+F-1, resident on the device."""
    from coeb_front import synth
    Tcw = np.stack([synth.motion_pose()] * F)
    if cfg.get("chain"):
        gray, boxes = synth.tracking_sequence(w, h, F, first=first)
        rgb, dep = synth.rgbd_from_gray(gray)
        bp.load_rgbd(rgb, dep, DEPTH_MAP_FACTOR, Tcw=Tcw)
        bp.set_frame_boxes(boxes[:, None, :])
        bp.host_frames = gray
        # what parity_check hands the oracle: the raw RGB-D input the device converted itself
        bp.bench_inputs = dict(first=first, rgb=rgb, dep=dep, boxes=boxes)
        return gray, Tcw
    frames = synth.make_frames(w, h, F, seed=1000, first=first)    # global frames first .. first+F-1
    dyn = dyn_batch(w, h, F, first) if cfg.get("dyn") else None
    bp.load(frames, Tcw=Tcw, dyn=dyn)
    bp.bench_inputs = dict(first=first, frames=frames, dyn=dyn)
    return frames, Tcw


def plan_pipelines(G, world, rank, pipelines, halo):
    """The bench's per-rank schedule: rank `rank`'s matched chunk of the G-frame sequence
    (dist.shard) split over up to `pipelines` contexts, each extracting the `halo` frames before
    its part.  Returns [(first global frame, frames extracted, frames counted)] per pipeline."""
    from coeb_front.dist import shard
    _, lo, hi = shard(G, world, rank)
    npipe = max(1, min(pipelines, hi - lo))
    subs = []
    for p in range(npipe):
        _, a, b = shard(hi - lo, npipe, p)
        f0 = max(lo + a - (halo - 1), 0)
        subs.append((f0, lo + b - f0 + 1, b - a))
    return subs


def make_pipelines(cfg, subs, device, streams=1, dry_run=False, rank=0):
    """One BatchPipeline per entry of plan_pipelines(), its synthetic input resident on the device
    (what rank_main times, and what tests/test_gpu_bench_scale.py checks against the oracle)."""
    bps = []
    try:
        for first_p, F_p, _ in subs:
            if dry_run:
                bpp = DryRunPipeline(rank)
            else:
                from coeb_front.pipeline import BatchPipeline
                bpp = BatchPipeline(cfg["w"], cfg["h"], F_p, nfeatures=cfg["nfeatures"], device=device)
            bps.append(bpp)
            bpp.ctx.set_batch_streams(streams)
            load_batch(bpp, cfg, cfg["w"], cfg["h"], F_p, first_p)
    except BaseException:
        for bpp in bps:
            bpp.close()
        raise
    return bps


def parity_picks(F, every=128):
    """Frames of a pipeline's batch that parity_check samples: the first three, both sides of the
    middle and of 1024, the last two, and every `every`-th frame."""
    picks = {0, 1, 2, F // 2 - 1, F // 2, F - 2, F - 1} | set(range(0, F, every))
    if F > 1024:
        picks |= {1023, 1024}
    return sorted(f for f in picks if 0 <= f < F)


def _oracle_checker():
    """The oracle module on its checker build (liborb_oracle.so, the build the tests use; the
    CPU-baseline legs switch the module to their timed builds and back)."""
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    O.LIB, O._lib = os.path.join(ROOT, "oracle", "liborb_oracle.so"), None
    return O


def _diff_kps(got, ref_kps, ref_desc):
    """Names of the fields in which a frame's device keypoints / descriptors differ from the oracle's."""
    if len(got["kps"]) != len(ref_kps):
        return ["count %d vs %d" % (len(got["kps"]), len(ref_kps))]
    bad = [f for f in got["kps"].dtype.names if not np.array_equal(got["kps"][f].view(np.uint32),
                                                                    ref_kps[f].view(np.uint32))]
    if len(ref_kps) and not np.array_equal(got["desc"], ref_desc):
        bad.append("descriptors (%d rows)" % int((got["desc"] != ref_desc).any(axis=1).sum()))
    return bad


def parity_check(bps, cfg, picks):
    """The oracle on sampled frames of the bench's own pipelines, after their last step (it runs
    after the timed region, in the CPU-baseline leg, and in tests/test_gpu_bench_scale.py).

    picks[p] lists pipeline p's batch-local frames.  Every field is compared bit for bit: the
    keypoint records (angles included) and descriptors, for f >= 1 the SearchByProjection count
    and match indices (th 15, 2*th retry below 20 matches, Tracking.cc:947-958), and for config D
    the whole configs[4] loop's per-frame records (bench.ChainCpu on frames f-3..f of the same
    pipeline, which is every dependency of frame f: dist.shard_frames).  Returns a summary dict."""
    O = _oracle_checker()
    from coeb_front import synth
    t0 = time.perf_counter()
    w, h, nf = cfg["w"], cfg["h"], cfg["nfeatures"]
    chain = bool(cfg.get("chain"))
    ex = O.Extractor(nf, 1.2, 8, 20, 7)
    cam = O.camera(ex, w, h, synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
    depth = synth.make_depth(w, h)
    I4 = np.eye(4, dtype=np.float32)
    Tc = synth.motion_pose()
    bad, nframes, nmatched = [], 0, 0
    for p, (bp, fl) in enumerate(zip(bps, picks)):
        inp = bp.bench_inputs
        cache = {}

        def extract(f):
            if f not in cache:
                fr = inp["frames"][f]
                cache[f] = ex.extract(fr, *inp["dyn"][f]) if inp["dyn"] is not None else ex.extract(fr)
            return cache[f]
        for f in fl:
            got = bp.frame(f, track=chain)
            nframes += 1
            tag = "pipeline %d frame %d (global %d)" % (p, f, inp["first"] + f)
            if chain:
                lo = max(0, f - 3)
                cl = ChainCpu(O, cfg, inp["rgb"][lo:f + 1], inp["dep"][lo:f + 1], inp["boxes"][lo:f + 1])
                cl.stride = bp.ctx.batch_results()[3]
                for i in range(f + 1 - lo):
                    cl.step(i)
                r, res = cl.last
            else:
                r, res = extract(f), None
            diff = _diff_kps(got, r["kps"], r["desc"])
            if f and not chain:
                prev = extract(f - 1)
                last = O.mapframe_from_extraction(prev["kps"], prev["desc"], depth, synth.TUM_FX, synth.TUM_FY,
                                                  synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
                ur, _ = O.stereo_from_rgbd(r["kps"], depth, synth.TUM_BF)
                nm, m = O.search_by_projection(cam, r["kps"], r["desc"], ur, last, Tc, I4, 15.0)
                if nm < 20:
                    nm, m = O.search_by_projection(cam, r["kps"], r["desc"], ur, last, Tc, I4, 30.0)
                res = dict(nmatches=nm, match=m)
            if f:
                nmatched += 1
                if got["nmatch"] != res["nmatches"] or not np.array_equal(got["match"], res["match"]):
                    diff.append("matches %d vs %d" % (got["nmatch"], res["nmatches"]))
            if f and chain:
                diff += _diff_track(got, res)
            if diff:
                bad.append("%s: %s" % (tag, ", ".join(diff)))
            if len(cache) > 8:
                for k in sorted(cache)[:-2]:
                    del cache[k]
    return dict(bit_exact=not bad, frames=nframes, matched_frames=nmatched, pipelines=len(bps),
                frames_per_pipeline=[len(fl) for fl in picks], mismatches=bad[:10], seconds=round(time.perf_counter() - t0, 2),
                compared="keypoint records (every field, angles bitwise), 256-bit descriptors, SearchByProjection "
                         "count + indices (th 15, retry 30)" + (", the configs[4] loop's T1 / nin1 / nmatchesMap / "
                                                                 "local matches / T / inliers / outliers / state"
                                                                 if chain else "") + " vs the oracle")


def _diff_track(got, res):
    """configs[4] per-frame records that differ (tests/test_gpu_parity.py::_check_chain's rules)."""
    d = []
    if not np.array_equal(got["T1"].view(np.uint32), np.asarray(res["T1"], np.float32).view(np.uint32)):
        d.append("T1")
    if got["nin1"] != res["nin1"]:
        d.append("nin1 %d vs %d" % (got["nin1"], res["nin1"]))
    if got["state"] != res["state"]:
        d.append("state %d vs %d" % (got["state"], res["state"]))
    if res["nmatches"] >= 20 and got["nmatches_map"] != res["nmatches_map"]:
        d.append("nmatchesMap")
    if res["state"] == 0:
        if got["ninliers"] != 0 or not np.array_equal(got["T"].view(np.uint32),
                                                       np.asarray(res["T1"], np.float32).view(np.uint32)):
            d.append("pose / inliers of an untracked frame")
        return d
    if got["nlocal"] != res["nlocal"] or not np.array_equal(got["local_match"], res["local_match"]):
        d.append("local matches %d vs %d" % (got["nlocal"], res["nlocal"]))
    if got["ninliers"] != res["ninliers"]:
        d.append("ninliers %d vs %d" % (got["ninliers"], res["ninliers"]))
    if not np.array_equal(got["T"].view(np.uint32), res["T"].view(np.uint32)):
        d.append("T")
    h2 = res["has2"] > 0
    if not np.array_equal(got["outlier"][h2], res["outlier"][h2]):
        d.append("outliers")
    return d


def dyn_batch(w, h, F, seed0=0):
    """Per-frame (boxes, T_M, blur_flag) of config 3: two boxes, 30 T_M points
    inside them and 30 outside, a fresh T_M draw per frame."""
    from coeb_front import synth
    return [synth.dynamic_inputs(w, h, seed=seed0 + f) for f in range(F)]


def level_pixels(w, h, nlevels=8, scale=1.2):
    s, tot = 1.0, 0
    for l in range(nlevels):
        if l:
            s = float(np.float32(np.float64(np.float32(s)) * np.float64(np.float32(scale))))
        inv = np.float32(1.0) / np.float32(s)
        tot += int(np.rint(np.float32(w) * inv)) * int(np.rint(np.float32(h) * inv))
    return tot


def fast_roi_pixels(w, h, nlevels=8, scale=1.2):
    """Pixels of the union of the FAST cell ROIs, [16, W_l-13) x [16, H_l-13) per level
    (ORBextractor.cc:795-798: minBorder = 16, maxBorder = W_l - 16 + 3)."""
    s, tot = 1.0, 0
    for l in range(nlevels):
        if l:
            s = float(np.float32(np.float64(np.float32(s)) * np.float64(np.float32(scale))))
        inv = np.float32(1.0) / np.float32(s)
        lw, lh = int(np.rint(np.float32(w) * inv)), int(np.rint(np.float32(h) * inv))
        tot += max(0, lw - 29) * max(0, lh - 29)
    return tot


# launches over the F - 1 consecutive frame pairs of a batch (the rest cover F frames)
PAIR_KERNELS = ("k_match", "k_gf_response", "k_gf_candidates", "k_gf_select", "k_subpix", "k_sharr", "k_lk", "k_fm",
                "k_pose", "k_track_prep", "k_tlm_pose_prep")
LK_WIN, LK_LEVELS = 22, 5          # calcOpticalFlowPyrLK(winSize 22x22, maxLevel 4), Frame.cc:335


def lk_level_sizes(w, h, levels=LK_LEVELS):
    out = [(w, h)]
    for _ in range(levels - 1):
        w, h = (w + 1) // 2, (h + 1) // 2
        out.append((w, h))
    return out


def kernel_bytes(name, w, h, nkp, nprev, npx, ncand, flow=None):
    """Algorithmic bytes of one launch per unit (each byte the algorithm must read or write,
    touched once), DESIGN.md s4.  The unit is a frame for the extraction / matching kernels and a
    frame pair for the ProcessMovingObject kernels (flow = per-pair means {keys, corners})."""
    flow = flow or {}
    corners, keys = flow.get("corners", 0.0), flow.get("keys", 0.0)
    lv = lk_level_sizes(w, h)
    if name == "k_rgbd_batch":  # RGB8 + 16U depth in, gray + 32F depth out
        return (3 + 2 + 1 + 4) * w * h
    if name == "k_gf_response":  # gray in, float Harris response out
        return 5 * w * h
    if name == "k_gf_candidates":  # response in, (value, index) keys out
        return 4 * w * h + 8 * keys
    if name == "k_gf_select":   # keys in, corners out
        return 8 * keys + 8 * corners
    if name == "k_subpix":      # per corner: the 24x24 source of the 23x23 interpolated window, point in/out
        return (24 * 24 + 16) * corners
    if name == "k_pyr_down":    # 4 launches: each frame's level l-1 in, level l out (mean per launch)
        return sum(a[0] * a[1] + b[0] * b[1] for a, b in zip(lv[:-1], lv[1:])) / (len(lv) - 1)
    if name == "k_sharr":       # every level of the previous frame in, short2 derivatives out
        return sum(x * y for x, y in lv) * (1 + 4)
    if name == "k_lk":          # per point and level: prev window, its derivatives, next window ((win+1)^2 px each)
        return corners * (LK_LEVELS * (LK_WIN + 1) ** 2 * (1 + 4 + 1) + 17)
    if name == "k_fm":          # points + status in, 3x3 SAD patches of both frames, T_M out
        return corners * (8 + 8 + 1 + 18 + 8)
    if name == "k_blur_flags":  # the box crop (120 x 160 px in config D)
        return 120 * 160
    if name in ("k_pose", "k_track_prep", "k_tlm_pose_prep"):   # per keypoint: MapPoint + keypoint + flags
        return (12 + 28 + 4 + 2) * nkp
    if name == "k_fast":        # read the FAST ROIs of every level, write candidate keys
        return fast_roi_pixels(w, h) + 4 * ncand
    if name == "k_blur":        # read + write every level
        return 2 * npx
    if name == "k_pyr_level":   # 7 launches: read level l-1, write level l (sum over launches / 7)
        return 2 * (npx - w * h) / 7.0 + w * h / 7.0
    if name == "k_octree":      # read candidates, write level keypoints
        return 4 * ncand + 4 * nkp
    if name == "k_describe":    # per keypoint: 749-px IC_Angle disc + 512 blurred samples in,
        return (749 + 512 + 4 + 60) * nkp   # key in, 28-B record + 32-B descriptor out
    if name == "k_match":       # read current kps+descs and LastFrame snapshot, write matches
        return 60 * nkp + (32 + 28 + 12 + 4) * nprev + 4 * nkp
    if name == "k_prep":
        return 28 * nkp + 4 * nkp + 25 * nkp
    return 0


def host_cpu_info():
    """CPU model (/proc/cpuinfo), the CPUs this process may run on (what `nproc` prints: the
    affinity mask) and the cgroup CPU quota if one is set (cpu.max), for the baseline record."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    cpus = sorted(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()
            if q != "max":
                quota = round(int(q) / int(period), 2)
    except (OSError, ValueError):
        pass
    return dict(cpu_model=model, nproc=len(cpus), cpu_quota=quota, machine_cpus=os.cpu_count()), cpus


def effective_cpus(info, cpus):
    """Threads the all-cores legs use: the affinity mask (`nproc`) capped by the cgroup CPU
    quota when one is set, so `cores` states the CPUs the run actually had."""
    n = len(cpus)
    if info.get("cpu_quota"):
        n = max(1, min(n, int(math.ceil(info["cpu_quota"]))))
    return n


def idle_cpus(cpus, k=3, window=0.5):
    """The k CPUs of the affinity mask that were idlest over `window` seconds (/proc/stat idle +
    iowait deltas), one per physical core where the topology says so: on a shared host cpus[0]
    can carry other load (round 4's driver run measured 44 frames/s single-thread where the
    builder's run on the same box type measured 79), so the single-thread legs run on measured-idle
    CPUs.  Returns [(cpu, idle_fraction)], idlest first."""
    def snap():
        st = {}
        try:
            with open("/proc/stat") as f:
                for ln in f:
                    if ln.startswith("cpu") and ln[3:4].isdigit():
                        v = ln.split()
                        nums = [int(x) for x in v[1:]]
                        st[int(v[0][3:])] = (nums[3] + (nums[4] if len(nums) > 4 else 0), sum(nums[:8]))
        except (OSError, ValueError):
            pass
        return st
    a = snap()
    time.sleep(window)
    b = snap()
    idle = []
    for c in cpus:
        if c in a and c in b and b[c][1] > a[c][1]:
            idle.append((c, (b[c][0] - a[c][0]) / (b[c][1] - a[c][1])))
    if not idle:
        return [(c, None) for c in cpus[:k]]
    idle.sort(key=lambda t: -t[1])

    def core_of(c):
        try:
            with open("/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list" % c) as f:
                return f.read().strip()
        except OSError:
            return str(c)
    out, cores = [], set()
    for c, fr in idle:
        if core_of(c) in cores:
            continue
        cores.add(core_of(c))
        out.append((c, round(fr, 3)))
        if len(out) == k:
            break
    return out


def _pinned_legs(run_leg, cpu_list, seconds):
    """run_leg(cpu, seconds) -> (median s/frame, frames) on each CPU of cpu_list (the timing thread
    pinned there); returns the median of the per-CPU medians and the per-CPU records."""
    per = []
    mask = os.sched_getaffinity(0)
    try:
        for c, fr in cpu_list:
            os.sched_setaffinity(0, {c})
            med, n = run_leg(c, seconds)
            per.append(dict(cpu=c, idle_before=fr, frames_per_s=round(1.0 / med, 3), frames=n))
    finally:
        os.sched_setaffinity(0, mask)
    vals = sorted(p["frames_per_s"] for p in per)
    return vals[len(vals) // 2], per


def _cpu_dyn(cfg, nfr):
    """Config C's per-frame dynamic-mask inputs (boxes, T_M, blur flags) for the CPU legs, as the
    device batch gets them (dyn_batch), or None."""
    return dyn_batch(cfg["w"], cfg["h"], nfr) if cfg.get("dyn") else None


def _single_thread_leg(O, lib_path, cfg, ex_args, frames, depth, cam, cpu, seconds, min_frames, warmup=20):
    """SURVEY.md s8(d)'s single-thread leg on one oracle build: `warmup` untimed frames, then
    extract (with config C's dynamic mask) + ComputeStereoFromRGBD + SearchByProjection (retry at
    2*th) per frame, median time."""
    from coeb_front import synth
    O.LIB = lib_path
    O._lib = None
    ex = O.Extractor(*ex_args)
    nfr = len(frames)
    dyn = _cpu_dyn(cfg, nfr)
    ext = (lambda i: ex.extract(frames[i % nfr], *dyn[i % nfr])) if dyn else (lambda i: ex.extract(frames[i % nfr]))
    Tc, Tl = synth.motion_pose(), np.eye(4, dtype=np.float32)
    prev = ext(0)
    for i in range(1, 1 + warmup):
        prev = ext(i)
    times = []
    t_end = time.perf_counter() + seconds
    i = 1 + warmup
    while (time.perf_counter() < t_end or len(times) < min_frames) and len(times) < 400:
        last = O.mapframe_from_extraction(prev["kps"], prev["desc"], depth, synth.TUM_FX, synth.TUM_FY,
                                          synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)   # map snapshot (untimed)
        t0 = time.perf_counter()
        r = ext(i)
        ur, _ = O.stereo_from_rgbd(r["kps"], depth, synth.TUM_BF)
        nm, _ = O.search_by_projection(cam, r["kps"], r["desc"], ur, last, Tc, Tl, 15.0)
        if nm < 20:
            O.search_by_projection(cam, r["kps"], r["desc"], ur, last, Tc, Tl, 30.0)
        times.append(time.perf_counter() - t0)
        prev = r
        i += 1
    return float(np.median(times)), len(times)


def cpu_baseline(cfg, seconds=9.0, min_frames=30):
    """Oracle ('port') timed on this host: extract + ComputeStereoFromRGBD + SearchByProjection
    (retry at 2*th) per frame, on consecutive synthetic frames.  The single-thread legs run
    pinned to one CPU (os.sched_setaffinity on the timing thread, SURVEY.md s8(d) `taskset -c`),
    20 warm-up frames each: the -O3 -march=native build (the reference's CMakeLists.txt:15 flags,
    auto-vectorised; the headline `value`) and a plain scalar build (-O3 -march=x86-64, no
    vectoriser) beside it.  The all-cores leg uses the -march=native build."""
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "native", "scalar"])
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from coeb_front import synth
    info, cpus = host_cpu_info()
    w, h = cfg["w"], cfg["h"]
    ex_args = (cfg["nfeatures"], 1.2, 8, 20, 7)
    depth = synth.make_depth(w, h)
    frames = synth.make_frames(w, h, 64, seed=5151)
    native = os.path.join(ROOT, "oracle", "liborb_oracle_native.so")
    scalar = os.path.join(ROOT, "oracle", "liborb_oracle_scalar.so")
    pick = idle_cpus(cpus, 3)
    try:
        O.LIB, O._lib = native, None
        cam = O.camera(O.Extractor(*ex_args), w, h, synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY,
                       synth.TUM_BF)
        val, per = _pinned_legs(lambda c, sec: _single_thread_leg(O, native, cfg, ex_args, frames, depth, cam, c, sec,
                                                                  min_frames), pick, seconds / len(pick))
        val_s, per_s = _pinned_legs(lambda c, sec: _single_thread_leg(O, scalar, cfg, ex_args, frames, depth, cam, c,
                                                                      sec, min_frames), pick, 0.6 * seconds / len(pick))
    finally:
        O.LIB, O._lib = native, None
    vals = [p["frames_per_s"] for p in per]
    out = dict(value=val, unit="frames/s", cores=1, kind="port",
               sample="single thread pinned to each of the %d idlest CPUs (%s; idle fraction measured over 0.5 s "
                      "before), per CPU >= %d consecutive %dx%d synthetic frames after 20 warm-up frames, oracle "
                      "(-O3 -march=native): extract%s + ComputeStereoFromRGBD + SearchByProjection (th 15, retry 30); "
                      "value = median of the per-CPU median frame rates"
                      % (len(pick), ", ".join(str(c) for c, _ in pick), min_frames, w, h,
                         " with the dynamic mask (2 boxes, 60 T_M points, blur flags per frame)" if cfg.get("dyn") else ""),
               spread=dict(min=min(vals), max=max(vals), per_cpu=per))
    out.update(info)
    out["caveat"] = CPU_CAVEAT
    vals_s = [p["frames_per_s"] for p in per_s]
    out["scalar_build"] = dict(value=val_s, unit="frames/s", cores=1, kind="port",
                               sample="the same legs on the plain scalar build (-O3 -march=x86-64 -fno-tree-vectorize "
                                      "-fno-tree-slp-vectorize), median of the per-CPU medians",
                               spread=dict(min=min(vals_s), max=max(vals_s), per_cpu=per_s))
    out["all_cores"] = cpu_baseline_parallel(O, cfg, frames, depth, cam, effective_cpus(info, cpus))
    return out


class ChainCpu:
    """The configs[4] loop on the oracle for one frame sequence (the CPU baseline of config D):
    per frame GrabImageRGBD's conversions, the Frame ctor (ProcessMovingObject against the
    previous gray frame, blur flags, masked extraction), ComputeStereoFromRGBD and track_frame
    (motion model + TrackLocalMap), and the frame's map snapshot for the next one."""

    def __init__(self, O, cfg, rgb, dep, boxes):
        from coeb_front import synth
        self.O, self.rgb, self.dep, self.boxes = O, rgb, dep, boxes
        self.ex = O.Extractor(cfg["nfeatures"], 1.2, 8, 20, 7)
        w, h = cfg["w"], cfg["h"]
        self.cam = O.camera(self.ex, w, h, synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
        self.isg = np.array(self.ex.p.inv_sigma2[:8], np.float32)
        self.stride = 8 * cfg["nfeatures"] + 256
        self.Tp = synth.motion_pose()
        self.state = None

    def step(self, i):
        from coeb_front import synth
        O = self.O
        g = O.image_to_gray(self.rgb[i])
        d = O.depth_to_float(self.dep[i], np.float32(DEPTH_MAP_FACTOR))
        b = self.boxes[i][None, :]
        if self.state is None:
            tm, bl = np.zeros((0, 2), np.float32), np.zeros(1, np.int32)
        else:
            tm = O.process_moving_object(self.state["gray"], g)
            tm = np.zeros((0, 2), np.float32) if tm is None else tm
            bl, _ = O.blur_flags(g, b)
        r = self.ex.extract(g, b, tm, bl)
        mf = O.mapframe_from_extraction(r["kps"], r["desc"], d, synth.TUM_FX, synth.TUM_FY, synth.TUM_CX,
                                        synth.TUM_CY, synth.TUM_BF)
        T1, res = np.eye(4, dtype=np.float32), None
        if self.state is not None:
            ur, _ = O.stereo_from_rgbd(r["kps"], d, synth.TUM_BF)
            res = O.track_frame(self.cam, self.isg, r, ur, self.state["mf"], self.state["mf_prev"], self.Tp,
                                self.state["T1"], self.stride, fx=synth.TUM_FX, fy=synth.TUM_FY, cx=synth.TUM_CX,
                                cy=synth.TUM_CY, bf=synth.TUM_BF)
            T1 = res["T1"]
        self.state = dict(gray=g, mf=mf, mf_prev=self.state["mf"] if self.state else None, T1=T1)
        self.last = (r, res)            # frame i's extraction and track_frame records (parity_check)


def cpu_chain_baseline(cfg, seconds=15.0, min_frames=20):
    """Config D's CPU baseline: ChainCpu (the oracle's full GrabImageRGBD loop) on consecutive
    frames of the same synthetic sequence, single thread pinned to one CPU, and all host cores
    frame-sequence-parallel (one sequence slice per thread)."""
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "native"])
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from coeb_front import synth
    O.LIB = os.path.join(ROOT, "oracle", "liborb_oracle_native.so")
    O._lib = None
    info, cpus = host_cpu_info()
    w, h = cfg["w"], cfg["h"]
    nfr = 64
    gray, boxes = synth.tracking_sequence(w, h, nfr, first=0)
    rgb, dep = synth.rgbd_from_gray(gray)
    def leg(cpu, sec):
        cl = ChainCpu(O, cfg, rgb, dep, boxes)
        for i in range(CHAIN_WARMUP):
            cl.step(i)
        times = []
        t_end = time.perf_counter() + sec
        i = CHAIN_WARMUP
        while (time.perf_counter() < t_end or len(times) < min_frames) and i < nfr:
            t0 = time.perf_counter()
            cl.step(i)
            times.append(time.perf_counter() - t0)
            i += 1
        return float(np.median(times)), len(times)
    pick = idle_cpus(cpus, 3)
    val, per = _pinned_legs(leg, pick, seconds / len(pick))
    vals = [p["frames_per_s"] for p in per]
    out = dict(value=val, unit="frames/s", cores=1, kind="port",
               sample="single thread pinned to each of the %d idlest CPUs (%s), per CPU >= %d consecutive %dx%d frames "
                      "of the synthetic tracking sequence after %d warm-up frames, oracle (-O3 -march=native): the full "
                      "GrabImageRGBD loop per frame (conversions, ProcessMovingObject, blur flags, masked extract, "
                      "stereo, motion model, TrackLocalMap); value = median of the per-CPU median frame rates"
                      % (len(pick), ", ".join(str(c) for c, _ in pick), min_frames, w, h, CHAIN_WARMUP),
               spread=dict(min=min(vals), max=max(vals), per_cpu=per))
    out.update(info)
    out["caveat"] = CPU_CAVEAT
    nthr = effective_cpus(info, cpus)
    import threading
    done = [0] * nthr
    t_stop = [0.0]

    def work(t):
        cl = ChainCpu(O, cfg, rgb, dep, boxes)
        j = (5 * t) % nfr
        while time.perf_counter() < t_stop[0]:
            cl.step(j)
            done[t] += 1
            j = (j + 1) % nfr
            if j == 0:
                cl.state = None                       # a new sequence: no predecessor
    t0 = time.perf_counter()
    t_stop[0] = t0 + 8.0
    ths = [threading.Thread(target=work, args=(t,)) for t in range(nthr)]
    for x in ths:
        x.start()
    for x in ths:
        x.join()
    dt = time.perf_counter() - t0
    out["all_cores"] = dict(value=round(sum(done) / dt, 3), unit="frames/s", cores=nthr, kind="port",
                            sample="%d threads (nproc capped by the cgroup quota) x 8 s, one oracle chain per thread on its own slice of the "
                                   "sequence; %d frames" % (nthr, sum(done)))
    return out


def cpu_baseline_parallel(O, cfg, frames, depth, cam, nthr, seconds=6.0):
    """SURVEY.md s8(d)'s all-cores frame-parallel CPU run: one oracle extractor per thread, each
    thread extracting + matching its own run of consecutive frames (ctypes calls release the GIL,
    and the oracle keeps no global state).  Threads = nproc, the CPUs this process may use."""
    import threading
    from coeb_front import synth
    Tc, Tl = synth.motion_pose(), np.eye(4, dtype=np.float32)
    nfr = len(frames)
    done = [0] * nthr
    t_end = [0.0]

    dyn = _cpu_dyn(cfg, nfr)

    def work(t):
        ex = O.Extractor(cfg["nfeatures"], 1.2, 8, 20, 7)
        ext = (lambda i: ex.extract(frames[i], *dyn[i])) if dyn else (lambda i: ex.extract(frames[i]))
        i = (7 * t) % nfr
        prev = ext(i)
        while time.perf_counter() < t_end[0]:
            i = (i + 1) % nfr
            last = O.mapframe_from_extraction(prev["kps"], prev["desc"], depth, synth.TUM_FX, synth.TUM_FY,
                                              synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
            r = ext(i)
            ur, _ = O.stereo_from_rgbd(r["kps"], depth, synth.TUM_BF)
            nm, _ = O.search_by_projection(cam, r["kps"], r["desc"], ur, last, Tc, Tl, 15.0)
            if nm < 20:
                O.search_by_projection(cam, r["kps"], r["desc"], ur, last, Tc, Tl, 30.0)
            done[t] += 1
            prev = r
    t0 = time.perf_counter()
    t_end[0] = t0 + seconds
    ths = [threading.Thread(target=work, args=(t,)) for t in range(nthr)]
    for x in ths:
        x.start()
    for x in ths:
        x.join()
    dt = time.perf_counter() - t0
    return dict(value=round(sum(done) / dt, 3), unit="frames/s", cores=nthr, kind="port",
                sample="%d threads (nproc capped by the cgroup quota) x %.0f s, one oracle extractor per thread, frame-parallel extract + "
                       "ComputeStereoFromRGBD + SearchByProjection (LastFrame snapshots inside the timed loop); "
                       "%d frames" % (nthr, seconds, sum(done)))


def cpu_extras(out, w, h, reps=5):
    """The oracle ('port', single thread) on the same extras calls as extras_timing: ms per
    call, for comparison with the device entry points (cpu_baseline leg only)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from coeb_front import synth
    kp0, d0 = out[0][0], out[0][1]
    kp1, d1 = out[1][0], out[1][1]
    z = np.float32(synth.DEPTH_Z)
    xw = np.stack([(kp0["x"] - np.float32(synth.TUM_CX)) * z / np.float32(synth.TUM_FX),
                   (kp0["y"] - np.float32(synth.TUM_CY)) * z / np.float32(synth.TUM_FY),
                   np.full(len(kp0), z, np.float32)], 1).astype(np.float32)
    ur1 = (kp1["x"] - np.float32(synth.TUM_BF) / z).astype(np.float32)
    ex = O.Extractor()
    cam = O.camera(ex, w, h, synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
    T = synth.motion_pose()
    res = {}

    def timed(name, fn):
        fn()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        res[name] = round((time.perf_counter() - t0) / reps * 1e3, 4)

    mp = synth.make_local_map(xw, d0, kp0["octave"], T, w, h, seed=1)
    timed("localmap_search_ms", lambda: O.search_local_map(cam, kp1, d1, ur1, np.full(len(kp1), -1, np.int32), mp,
                                                           3.0, 0.8))
    kf = synth.make_keyframe_points(xw, d0, kp0["octave"], kp0["angle"], seed=1)
    timed("relocalisation_search_ms", lambda: O.search_keyframe(cam, kp1, d1, None, kf, T, 10.0, 100, True))
    P = synth.make_pose_problem(n=len(kp1), seed=1)
    isg = np.array([1.0 / (1.2 ** (2 * l)) for l in range(8)], np.float32)
    timed("pose_optimization_ms", lambda: O.pose_optimization(P["kps"], P["has_mp"], P["xw"], P["ur"], isg,
                                                              synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY,
                                                              synth.TUM_BF, P["Tcw_init"]))
    prev, cur, _ = synth.moving_object_pair(640, 480, 0)
    timed("process_moving_object_ms", lambda: O.process_moving_object(prev, cur))
    return res


def _pmc_file(stem, w, h, tag=None):
    """The committed PMC summary collected at frame size w x h: profiles/<stem>_<tag>.json for a
    config with its own kernels (tag "D": the configs[4] loop), else profiles/<stem>.json (config
    A's 640x480) or profiles/<stem>_<w>x<h>.json; None when none matches the size."""
    names = ("%s_%s.json" % (stem, tag),) if tag else ("%s.json" % stem, "%s_%dx%d.json" % (stem, w, h))
    for name in names:
        try:
            with open(os.path.join(ROOT, "profiles", name)) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if (d.get("width"), d.get("height")) == (w, h):
            d["_file"] = "profiles/" + name
            return d
    return None


def pmc_traffic(kernel, frames_per_launch, w, h, tag=None):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, written by tools/pmc_summary.py --json from separate
    FETCH_SIZE / WRITE_SIZE passes of this bench), scaled to this run's frames per launch.
    None unless the counters were collected at this frame size."""
    try:
        d = _pmc_file("pmc_traffic", w, h, tag)
        if d is None:
            return None, None
        k = d["kernels"][kernel]
        return (int(k["traffic_bytes"] * frames_per_launch / d["frames_per_launch"]),
                "%s (%s)" % (d["_file"], d.get("command", "")))
    except (OSError, KeyError, ValueError, ZeroDivisionError):
        return None, None


def pmc_valu(kernel, w, h, tag=None):
    """VALU issue utilisation of `kernel` from the committed PMC summary (profiles/pmc_valu.json,
    tools/pmc_summary.py --valu-json: SQ_INSTS_VALU / (2 x 256 CUs x busy cycles)), if collected
    at this frame size."""
    try:
        d = _pmc_file("pmc_valu", w, h, tag)
        if d is None:
            return None
        k = d["kernels"][kernel]
        out = dict(valu_issue_frac=k["valu_issue_frac"], valu_insts_per_launch=k["valu_insts"],
                   source="%s (%s)" % (d["_file"], d.get("command", "")))
        for key in ("wait_inst_frac", "wait_any_frac", "lds_conflict_per_lds_inst"):
            if key in k:
                out[key] = k[key]
        return out
    except (OSError, KeyError, ValueError):
        return None


class DryRunPipeline:
    """CPU stand-in with the BatchPipeline surface, for testing bench's multi-rank plumbing."""

    class _Ctx:
        def __init__(self):
            self._on = False

        def profile(self, on=True):
            self._on = on

        def profile_reset(self):
            pass

        def profile_read(self):
            return {"k_fast": (1.0, 1)} if self._on else {}

        def debug_read(self, what, f=0):
            return np.zeros(4, np.uint8)

        def set_batch_streams(self, n):
            pass

    def __init__(self, rank):
        self.rank = rank
        self.ctx = self._Ctx()

    def load(self, frames, **kw):
        self.F = len(frames)

    def load_rgbd(self, images, depth, factor, **kw):
        self.F = len(images)

    def set_frame_boxes(self, boxes):
        pass

    def run(self, **kw):
        time.sleep(0.002 * (1 + self.rank))   # ranks finish at different times: max must win

    def synchronize(self):
        pass

    def results(self):
        from coeb_front import KEYPOINT_DTYPE
        out = [(np.zeros(1000, KEYPOINT_DTYPE), np.zeros((1000, 32), np.uint8))] * self.F
        return out, None, [None] + [750] * (self.F - 1)

    def close(self):
        pass


def extras_timing(ctx, out, w, h, reps=20):
    """Per-call wall time of the host-buffer entry points beyond the headline path (SURVEY.md
    s8(f) rows 2-4), on inputs built from the batch's own extraction of frames 0 and 1: mean
    ms per call including the PCIe copies and the synchronisation each call performs."""
    import coeb_front as cf
    from coeb_front import synth
    kp0, d0 = out[0][0], out[0][1]
    kp1, d1 = out[1][0], out[1][1]
    z = np.float32(synth.DEPTH_Z)
    xw = np.stack([(kp0["x"] - np.float32(synth.TUM_CX)) * z / np.float32(synth.TUM_FX),
                   (kp0["y"] - np.float32(synth.TUM_CY)) * z / np.float32(synth.TUM_FY),
                   np.full(len(kp0), z, np.float32)], 1).astype(np.float32)
    ur1 = (kp1["x"] - np.float32(synth.TUM_BF) / z).astype(np.float32)
    cam = cf.make_camera(synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF, w, h)
    T = synth.motion_pose()
    res = {}

    def timed(name, fn, note):
        fn()
        t0 = time.perf_counter()
        for _ in range(reps):
            r = fn()
        res[name] = dict(ms_per_call=round((time.perf_counter() - t0) / reps * 1e3, 4), result=int(r), note=note)

    mp = synth.make_local_map(xw, d0, kp0["octave"], T, w, h, seed=1)
    lm = cf.LocalMap(mp["in_view"], mp["proj_x"], mp["proj_y"], mp["proj_xr"], mp["level"], mp["view_cos"],
                     mp["descriptor"], mp["observations"])
    F1 = cf.Frame(kp1, d1, ur1)
    m = cf.ORBmatcher(0.8, ctx=ctx)
    timed("localmap_search", lambda: m.SearchByProjection(cf.Frame(kp1, d1, ur1), lm, 3.0, camera=cam),
          "SearchByProjection(F, %d local-map points, th 3), %d keypoints" % (lm.N, F1.N))
    kf = synth.make_keyframe_points(xw, d0, kp0["octave"], kp0["angle"], seed=1)
    kfp = cf.KeyFramePoints(kf["valid"], kf["world_pos"], kf["descriptor"], kf["max_distance"], kf["min_distance"],
                            kf["angle"])
    mk = cf.ORBmatcher(0.75, True, ctx=ctx)
    timed("relocalisation_search",
          lambda: mk.SearchByProjection(cf.Frame(kp1, d1, ur1, Tcw=T), kfp, set(), 10.0, 100, cam),
          "SearchByProjection(F, KeyFrame of %d points, th 10, ORBdist 100)" % kfp.N)
    P = synth.make_pose_problem(n=len(kp1), seed=1)

    def pose():
        Fp = cf.Frame(P["kps"], np.zeros((len(P["kps"]), 32), np.uint8), P["ur"], Tcw=P["Tcw_init"])
        Fp.mvpMapPoints = np.where(P["has_mp"] > 0, 0, -1).astype(np.int32)
        Fp.mvMapPointPos = P["xw"]
        return cf.Optimizer.PoseOptimization(Fp, cam, ctx)
    timed("pose_optimization", pose, "PoseOptimization, %d edges (20 %% gross outliers), 4 x 10 LM iterations"
          % int(P["has_mp"].sum()))
    dist = (0.262383, -0.953104, -0.005358, 0.002628, 1.163314)
    timed("undistort_keypoints", lambda: len(cf.UndistortKeyPoints(ctx, kp1, cam, dist)),
          "UndistortKeyPoints, %d keypoints, TUM1 distortion" % len(kp1))
    prev, cur, _ = synth.moving_object_pair(640, 480, 0)
    timed("process_moving_object", lambda: len(cf.ProcessMovingObject(ctx, prev, cur)),
          "ProcessMovingObject 640x480 (goodFeaturesToTrack 1000, cornerSubPix, 5-level LK, RANSAC F), "
          "result = |T_M|")
    return res


def config5_timing(bp, batch, steps=10):
    """BASELINE configs[4] on the same batch: extract + match + TrackWithMotionModel's
    PoseOptimization for every matched frame, device-resident like `value`."""
    bp.run(pose=True)
    bp.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        bp.run(pose=True)
    bp.synchronize()
    dt = time.perf_counter() - t0
    _, nin, _ = bp.pose_results()
    return dict(value=round(batch * steps / dt, 2), unit="frames/s", ms_per_step=round(dt / steps * 1e3, 4),
                steps=steps, tracked_frames=int(sum(1 for x in nin[1:] if x > 0)),
                inliers_per_frame=round(float(np.mean(nin[1:])), 1),
                note="extract + SearchByProjection + PoseOptimization per frame (bench.py --config D for the full line)")


def config3_timing(bp, frames, Tcw, w, h, batch, steps=10):
    """BASELINE configs[2] on the same batch: extract with the dynamic mask (boxes, T_M,
    blur_flag per frame) + depth association + match, device-resident like `value`."""
    bp.load(frames, Tcw=Tcw, dyn=dyn_batch(w, h, batch + 1))
    bp.run()
    bp.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        bp.run()
    bp.synchronize()
    dt = time.perf_counter() - t0
    out, _, nms = bp.results()
    return dict(value=round(batch * steps / dt, 2), unit="frames/s", ms_per_step=round(dt / steps * 1e3, 4),
                steps=steps, keypoints_per_frame=round(float(np.mean([len(o[0]) for o in out[1:]])), 1),
                matches_per_frame=round(float(np.mean(nms[1:])), 1),
                note="640x480, 2 boxes + 60 T_M points + blur_flag [0,1] per frame (bench.py --config C for the full line)")


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs to drive.  Under torch.distributed.run this must equal WORLD_SIZE (one process "
                         "per GPU); started directly, bench drives devices 0..N-1 from N host threads")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None,
                    help="matched frames per step per GPU (weak scaling; default: the config's batch)")
    ap.add_argument("--global-frames", type=int, default=None,
                    help="fixed number of matched frames per step, sharded over the GPUs with one halo frame "
                         "each (strong scaling; config B defaults to BASELINE configs[3]'s 512)")
    ap.add_argument("--pipelines", type=int, default=None,
                    help="independent batch pipelines (contexts) per GPU whose kernels overlap (default: the "
                         "config's); the GPU's batch is split between them, each with its own halo frame")
    ap.add_argument("--config", default="A", choices=sorted(CONFIGS))
    ap.add_argument("--side-stream", default=None, choices=("own", "shared", "off"),
                    help="extraction side stream per pipeline (own), one per GPU shared by the pipelines "
                         "(shared), or none (off); default: the config's")
    ap.add_argument("--streams", type=int, default=1,
                    help="HIP streams the batch is chunked over (kernels of different chunks overlap)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="skip HIP-event kernel timing")
    ap.add_argument("--no-e2e", action="store_true", help="skip the PCIe-inclusive host-buffer measurement")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the per-call timing of the other entry points (local map, relocalisation, pose)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: exercise the rank/timing/JSON plumbing with a stand-in pipeline (tests)")
    return ap.parse_args(argv)


def main():
    args = parse_args()
    if args.global_frames is None and args.config == "B":
        args.global_frames = 512
    if args.batch is None:
        args.batch = CONFIGS[args.config].get("batch", 256)
    if args.pipelines is None:
        args.pipelines = CONFIGS[args.config].get("pipelines", 1)
    # read by each context when it first extracts (csrc/coeb_capi.hip side_stream).  The config's
    # default only adds the shared stream; an explicit --side-stream also overrides the environment
    # (the PMC / profiling passes export COEB_SIDE_STREAM=0 and pass no --side-stream)
    explicit = args.side_stream is not None
    if not explicit:
        args.side_stream = CONFIGS[args.config].get("side_stream", "own")
    if args.side_stream == "shared":
        os.environ["COEB_SIDE_SHARED"] = "1"
        if explicit:
            os.environ["COEB_SIDE_STREAM"] = "1"
    elif args.side_stream == "off":
        os.environ["COEB_SIDE_STREAM"] = "0"
    elif explicit:
        os.environ["COEB_SIDE_SHARED"] = "0"
        os.environ["COEB_SIDE_STREAM"] = "1"
    if CONFIGS[args.config].get("side_eager") and "COEB_SIDE_EAGER" not in os.environ:
        os.environ["COEB_SIDE_EAGER"] = "1"      # read by coeb_create
    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    if env_world > 1 or "LOCAL_RANK" in os.environ:
        # one process per GPU under torch.distributed.run
        if env_world != args.gpus:
            sys.exit("bench.py: --gpus %d but WORLD_SIZE=%d: refusing to report a run on a different number "
                     "of GPUs" % (args.gpus, env_world))
        from coeb_front.dist import Ranks
        ranks = Ranks()
        if not args.dry_run:
            check_devices(1 if ONE_DEVICE else ranks.local_rank + 1)
        rank_main(ranks, args)
        return
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if not args.dry_run:
        check_devices(1 if ONE_DEVICE else args.gpus)
    if args.gpus == 1:
        from coeb_front.dist import Ranks
        rank_main(Ranks(), args)
        return
    # N devices from N host threads of this process (no torch.cuda anywhere)
    import threading
    from coeb_front.dist import ThreadRanks
    grp = ThreadRanks(args.gpus)
    errors = []

    def body(r):
        try:
            rank_main(grp.view(r), args)
        except BaseException as e:   # noqa: BLE001 - reported below, the process exits non-zero
            errors.append((r, e))
            grp.abort()
    ths = [threading.Thread(target=body, args=(r,), name="rank%d" % r) for r in range(args.gpus)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    if errors:
        import traceback
        for r, e in sorted(errors, key=lambda x: x[0]):
            print("rank %d failed:" % r, file=sys.stderr)
            traceback.print_exception(type(e), e, e.__traceback__)
        sys.exit(1)


def check_devices(n):
    import coeb_front
    have = coeb_front.lib().coeb_device_count()
    if have < n:
        sys.exit("bench.py: %d GPU(s) requested but only %d visible" % (n, have))


def rank_main(ranks, args):
    world, rank, local_rank = ranks.world, ranks.rank, ranks.local_rank
    if ONE_DEVICE:
        local_rank = 0          # rehearsal: every rank's context on device 0
    from coeb_front import synth
    from coeb_front.dist import shard_frames
    cfg = CONFIGS[args.config]
    w, h = cfg["w"], cfg["h"]
    strong = args.global_frames is not None
    G = args.global_frames if strong else args.batch * world       # matched frames per step, all ranks
    if G < world:
        raise SystemExit("bench.py: %d matched frames cannot be split over %d GPUs" % (G, world))
    chain = bool(cfg.get("chain"))
    halo = 3 if chain else 1
    _, nmatched = shard_frames(G, world, rank, halo=halo)[1:]
    # the rank's matched chunk split over its pipelines, each extracting its own halo
    subs = plan_pipelines(G, world, rank, args.pipelines, halo)
    npipe = len(subs)
    bps = make_pipelines(cfg, subs, local_rank, args.streams, args.dry_run, rank)
    Tcw = np.stack([synth.motion_pose()] * subs[0][1])
    bp = bps[0]                         # results, roofline pass, extras and the PCIe leg use pipeline 0
    first, F, nmatched0 = subs[0]
    # every rank states what it covers; the sum must be the whole sequence
    covered = int(ranks.sum(nmatched))
    if covered != G:
        raise RuntimeError("shards cover %d of %d matched frames" % (covered, G))
    per_rank = [shard_frames(G, world, r, halo=halo)[2] for r in range(world)]

    kw = step_kwargs(cfg)
    for _ in range(args.warmup):
        for bpp in bps:
            bpp.run(**kw)
    for bpp in bps:
        bpp.synchronize()
    out, matches, nms = bp.results()
    c0 = F - nmatched0                                              # first counted frame of the batch
    nkp = float(np.mean([len(o[0]) for o in out[c0:]]))
    nmatch = float(np.mean(nms[c0:]))
    ncand = int(bp.ctx.debug_read("cand_n", 1).view(np.int32).sum())
    flow = None
    if chain and not args.dry_run:        # per-pair Harris keys / corners of ProcessMovingObject
        fc = bp.ctx.debug_read("flow_counts").view(np.int32).reshape(-1, 2)[c0 - 1:]
        flow = dict(keys=float(fc[:, 0].mean()), corners=float(fc[:, 1].mean()))
    tracking = None
    if chain and not args.dry_run:
        tr = bp.track_results()
        st = tr["state"][c0:]
        tracking = dict(frames=len(st), tracked=st.count(2), local_map_failed=st.count(1), motion_model_failed=st.count(0),
                        inliers_per_frame=round(float(np.mean(tr["ninliers"][c0:])), 1),
                        local_map_matches_per_frame=round(float(np.mean(tr["nlocal"][c0:])), 1),
                        motion_model_matches_map_per_frame=round(float(np.mean(tr["nmatches_map"][c0:])), 1))

    # timed region: no instrumentation (HIP event pairs around every launch cost ~10 us each)
    ranks.barrier()
    for bpp in bps:
        bpp.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        for bpp in bps:                  # enqueue only: the pipelines' kernels overlap on the device
            bpp.run(**kw)
    for bpp in bps:
        bpp.synchronize()
    t1 = time.perf_counter()
    ranks.barrier()
    elapsed = ranks.max(t1 - t0)

    # per-kernel device time (rank 0): a separate pass with HIP events, kernels serialised on
    # one stream so each event pair brackets exactly one launch
    prof = {}
    prof_steps = 0
    if not args.no_profile and rank == 0:
        prof_steps = max(1, min(args.steps, 10))
        bp.ctx.set_batch_streams(1)
        bp.ctx.profile(True)
        bp.ctx.profile_reset()
        for _ in range(prof_steps):
            bp.run(**kw)
            if chain:
                # the configs[4] loop runs PoseOptimization / TrackLocalMap on a pose stream that
                # overlaps the next step's conversion and flow kernels: join it, so every event
                # pair brackets a launch with nothing else on the device
                bp.synchronize()
        bp.synchronize()
        prof = bp.ctx.profile_read()
        bp.ctx.profile(False)
        bp.ctx.set_batch_streams(args.streams)
    ranks.barrier()


    value = G * args.steps / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    if rank == 0:
        npx = level_pixels(w, h)
        roof = None
        tag = "D" if chain else None
        if prof:
            dom = max(prof.items(), key=lambda kv: kv[1][0])
            name, (tot_ms, launches) = dom
            avg_s = tot_ms / launches / 1e3
            frames_per_launch = F - 1 if name in PAIR_KERNELS else F
            # achieved = SURVEY.md s8(d)'s algorithmic bytes per frame (W*H + 60 N_kp + 36 N_prev) x
            # the frames the launch processes / the launch's average duration; the kernel's own
            # touched-once bytes are reported beside it as `kernel_own`
            bpl = (w * h + 60 * nkp + 36 * nkp) * frames_per_launch
            achieved = bpl / avg_s / 1e9
            own = kernel_bytes(name, w, h, nkp, nkp, npx, ncand, flow) * frames_per_launch
            traffic, tsrc = pmc_traffic(name, frames_per_launch, w, h, tag)
            roof = dict(bound="hbm", achieved=round(achieved, 3), peak=HBM_PEAK_GBS, unit="GB/s",
                        frac=round(achieved / HBM_PEAK_GBS, 6), traffic=traffic, kernel=name,
                        avg_launch_us=round(avg_s * 1e6, 2), bytes_per_launch=int(bpl),
                        bytes_rule="SURVEY.md s8(d): (W*H + 60*N_kp + 36*N_prev) x %d frames" % frames_per_launch,
                        kernel_own=dict(bytes_per_launch=int(own), achieved=round(own / avg_s / 1e9, 3),
                                        frac=round(own / avg_s / 1e9 / HBM_PEAK_GBS, 6)))
            if name not in IMAGE_KERNELS:
                # a dominant kernel that reads no image (config D's k_pose): the headline figures are
                # its own bytes, and the s8(d) image-byte figure moves aside
                roof.update(achieved=roof["kernel_own"]["achieved"], frac=roof["kernel_own"]["frac"],
                            bytes_per_launch=int(own),
                            bytes_rule="%s's own touched-once bytes x %d frames (DESIGN.md s4); the kernel "
                                       "reads no image, so SURVEY.md s8(d)'s image bytes do not apply"
                                       % (name, frames_per_launch),
                            s8d=dict(bytes_per_launch=int(bpl), achieved=round(achieved, 3),
                                     frac=round(achieved / HBM_PEAK_GBS, 6)))
            if traffic is not None:
                roof["traffic_source"] = tsrc
            # the kernel is bound by integer VALU issue, not HBM: the PMC VALU fraction says how
            # close it runs to the chip's issue ceiling (2 wave64 VALU instructions per CU per cycle)
            valu = pmc_valu(name, w, h, tag)
            if valu is not None:
                roof["valu"] = valu
        pipeline_bytes = w * h + 60 * nkp + 36 * nkp     # B = W*H + 60 N_kp + 36 N_prev
        line = dict(metric=METRIC, value=round(value, 2), unit="frames/s", n_gpus=world, steps=args.steps,
                    warmup=args.warmup, ms_per_step=round(ms_per_step, 4), higher_is_better=True,
                    scaling="strong" if strong else "weak", vs_baseline=None, dtype="u8",
                    data=cfg.get("data", "synthetic (TUM-like rectangles + noise, (+2,+1) px/frame, Z=2 m)"),
                    config=dict(workload=cfg["workload"], width=w, height=h, nfeatures=cfg["nfeatures"],
                                nlevels=8, matched_frames_per_step=G, frames_per_rank=per_rank,
                                halo_frames_per_rank=halo, pipelines_per_gpu=npipe,
                                frames_per_pipeline=[sp[2] for sp in subs], streams_per_gpu=args.streams,
                                ranks="threads" if isinstance(ranks, _thread_rank_type()) else
                                      ("processes" if world > 1 else "single"),
                                parallelism="frame-sharded x%d (no collectives)" % world,
                                hw_queues=int(HW_QUEUES) if HW_QUEUES and HW_QUEUES.isdigit() else
                                          "GPU_MAX_HW_QUEUES unset (HIP default 4)",
                                side_stream="off" if os.environ.get("COEB_SIDE_STREAM", "1")[:1] == "0" else
                                            ("shared" if os.environ.get("COEB_SIDE_SHARED", "0")[:1] == "1"
                                             else "own"),
                                side_stream_created="with the context" if os.environ.get("COEB_SIDE_EAGER", "0")[:1] == "1"
                                                    else "at the first extraction"),
                    roofline=roof,
                    pipeline_roofline=dict(bytes_per_frame=int(pipeline_bytes),
                                           achieved_GBps=round(value * pipeline_bytes / 1e9, 3),
                                           frac=round(value * pipeline_bytes / 1e9 / HBM_PEAK_GBS / world, 6)),
                    kernels_ms_per_step={k: round(v[0] / max(1, prof_steps), 4) for k, v in prof.items()},
                    kernels_profiled_steps=prof_steps,
                    kernels_note="ms per launch set of pipeline 0 alone (%d frames), side stream off, HIP events on "
                                 "the context stream; the step runs %d such pipelines concurrently" % (F, npipe),
                    keypoints_per_frame=round(nkp, 1), matches_per_frame=round(nmatch, 1),
                    pcie_inclusive=None)
        if tracking is not None:
            line["tracking"] = tracking
        if flow is not None:
            line["flow_per_pair"] = dict(harris_keys=round(flow["keys"], 1), corners=round(flow["corners"], 1))
        if ONE_DEVICE and world > 1:
            line["rehearsal_one_device"] = True
        if not args.no_cpu_baseline and world == 1 and not args.dry_run:
            # the timed pipelines' own outputs (their last step) against the oracle, before the
            # extras below reload pipeline 0: 4 frames of pipeline 0, every field bit for bit
            line["parity_sample"] = parity_check([bp], cfg, [[1, 2, F // 2, F - 1]])
        if not args.no_extras and world == 1 and not args.dry_run:
            line["extras"] = extras_timing(bp.ctx, out, w, h)
            # the one-frame-at-a-time legs run their calling thread on the idlest CPU, as the CPU
            # baseline's single-thread legs do: on the shared host a busy core adds tens of us of
            # jitter to a 0.3 ms call sequence (the C++ child inherits the affinity)
            sf_cpu = idle_cpus(sorted(os.sched_getaffinity(0)), k=1)[0][0]
            mask = os.sched_getaffinity(0)
            try:
                os.sched_setaffinity(0, {sf_cpu})
                line["extras"]["single_frame"] = single_frame_timing(w, h)
                line["extras"]["single_frame_cpp"] = single_frame_cpp(w, h)
            finally:
                os.sched_setaffinity(0, mask)
            for k in ("single_frame", "single_frame_cpp"):
                line["extras"][k]["cpu"] = sf_cpu
            if not cfg.get("dyn") and not cfg.get("pose") and not chain:
                line["extras"]["config5_tracking"] = config5_timing(bp, nmatched0)
                line["extras"]["config3_dynamic_mask"] = config3_timing(bp, synth.make_frames(w, h, F, seed=1000),
                                                                        Tcw, w, h, nmatched0)
        if not args.no_cpu_baseline and world == 1 and not args.dry_run:
            cb = cpu_chain_baseline(cfg) if chain else cpu_baseline(cfg)
            if "extras" in line:
                cb["extras_ms_per_call"] = cpu_extras(out, w, h)
            line["cpu_baseline"] = cb
            line["speedup_vs_cpu_baseline"] = round(value / cb["value"], 1)
    # PCIe-inclusive leg last, with the device-resident pipeline closed: its two contexts and copy
    # queue then have hardware queues of their own
    host_frames, host_tcw = getattr(bp, "host_frames", None), getattr(bp, "Tcw", None)
    for bpp in bps:
        bpp.close()
    e2e = None
    g0 = int(ranks.sum(nmatched0))      # the PCIe leg streams pipeline 0's batch on every rank
    if not args.no_e2e and not args.dry_run and not chain:
        e2e = e2e_timing(host_frames, host_tcw, ranks, g0, 30, cfg, local_rank)
    if rank == 0:
        line["pcie_inclusive"] = e2e
        print(json.dumps(line), flush=True)
    ranks.close()


def _thread_rank_type():
    from coeb_front.dist import _ThreadRank
    return _ThreadRank


def e2e_timing(frames, Tcw, ranks, G, steps, cfg, device):
    """PCIe-inclusive rate (reported, never `value`): gray frames start in page-locked host
    memory, keypoints / descriptors / counts / matches end in page-locked host memory.
    HostStream's ring mode: uploads of later batches overlap the current batch's kernels and
    downloads."""
    from coeb_front import HostBuffer
    from coeb_front.pipeline import HostStream
    F, H, W = frames.shape
    hs = HostStream(W, H, F, nfeatures=cfg["nfeatures"], device=device, Tcw=Tcw)
    src = HostBuffer(F * H * W)
    src.view(np.uint8, (F, H, W))[:] = frames
    try:
        for i in range(4):                    # warm-up: both slots twice
            hs.submit(i, src)
        hs.wait(2)
        hs.wait(3)
        ranks.barrier()
        te0 = time.perf_counter()
        for i in range(steps):               # device-side ordering only: the host never blocks here
            hs.submit(i, src)
        hs.wait(steps - 2)
        hs.wait(steps - 1)
        te = ranks.max(time.perf_counter() - te0)
        out, _, nms = hs.results(steps - 1)
        ok = len(out) == F and sum(len(o[0]) for o in out) > 0
    finally:
        hs.close()
        src.free()
    return dict(value=round(G * steps / te, 2), unit="frames/s", ms_per_step=round(te / steps * 1e3, 4), steps=steps,
                results_nonempty=bool(ok),
                note="gray frames uploaded from page-locked host memory and keypoints/descriptors/counts/matches "
                     "downloaded to page-locked host memory every step (HostStream ring mode: an upload queue "
                     "filling three device input buffers back to back beside the kernels; results downloaded "
                     "on the compute stream)")


def single_frame_timing(w, h, reps=50, warm=5):
    """Drop-in latency of one frame from host buffers, as the sequential Tracking thread calls it
    (Tracking.cc:229 -> Frame ctor -> ExtractORB; ComputeStereoFromRGBD; TrackWithMotionModel's
    SearchByProjection, Tracking.cc:947-958): coeb_extract + coeb_stereo_from_rgbd +
    coeb_match_lastframe (th 15, retry 30 below 20 matches), frame i matched against frame i-1's
    extraction (its MapPoint snapshot -- world positions from its depth, its descriptors -- is the
    Tracking state the adapter packs, built before the timer starts).  Median ms per frame, and
    the median of each call."""
    import ctypes as C
    import coeb_front as cf
    from coeb_front import synth
    ctx = cf.Context(max_width=w, max_height=h, max_batch=1)
    try:
        fr = synth.make_frames(w, h, reps + warm + 1, seed=77)
        depth = synth.make_depth(w, h)
        cam = cf.make_camera(synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF, w, h)
        m = cf.ORBmatcher(0.9, True, ctx=ctx)
        Tc, Tl = synth.motion_pose(), np.eye(4, dtype=np.float32)

        stereo_fn, dptr, bf = cf.lib().coeb_stereo_from_rgbd, depth.ctypes.data, C.c_float(synth.TUM_BF)

        def stereo(k):
            ur = np.empty(len(k), np.float32)
            dep = np.empty(len(k), np.float32)
            ctx.check(stereo_fn(ctx.h, k.ctypes.data, len(k), dptr, w, h, w, bf, ur.ctypes.data, dep.ctypes.data))
            return ur, dep

        def snapshot(k, d, z):
            xw = np.stack([(k["x"] - np.float32(synth.TUM_CX)) * z / np.float32(synth.TUM_FX),
                           (k["y"] - np.float32(synth.TUM_CY)) * z / np.float32(synth.TUM_FY), z], 1).astype(np.float32)
            return cf.Frame(k, d, Tcw=Tl, map_points=dict(world_pos=xw, descriptor=d,
                                                          observations=np.full(len(k), 2, np.int32),
                                                          valid=(z > 0).astype(np.uint8)))
        k, d = ctx.extract(fr[0])
        last = snapshot(k, d, stereo(k)[1])
        times, parts, nms = [], [], []
        for i in range(1, reps + warm + 1):
            t0 = time.perf_counter()
            k, d = ctx.extract(fr[i])
            t1 = time.perf_counter()
            ur, dep = stereo(k)
            t2 = time.perf_counter()
            cur = cf.Frame(k, d, ur, Tcw=Tc)
            nm = m.SearchByProjection(cur, last, 15.0, False, cam)
            if nm < 20:                                                # Tracking.cc:954-958
                cur = cf.Frame(k, d, ur, Tcw=Tc)
                nm = m.SearchByProjection(cur, last, 30.0, False, cam)
            t3 = time.perf_counter()
            if i > warm:
                times.append(t3 - t0)
                parts.append((t1 - t0, t2 - t1, t3 - t2))
                nms.append(nm)
            last = snapshot(k, d, dep)                                  # untimed: the Tracking state
        med = np.median(np.array(parts), axis=0) * 1e3
        return dict(ms_per_frame=round(float(np.median(times)) * 1e3, 4), reps=reps,
                    matches=int(np.median(nms)), min_matches=int(min(nms)),
                    ms_extract=round(float(med[0]), 4), ms_stereo=round(float(med[1]), 4),
                    ms_match=round(float(med[2]), 4),
                    note="median over %d consecutive frames (after %d warm-up frames) of coeb_extract + "
                         "coeb_stereo_from_rgbd + coeb_match_lastframe (th 15, retry 30) from host buffers, frame i "
                         "matched against frame i-1's extraction (one frame at a time, synchronous, as the Tracking "
                         "thread)" % (reps, warm))
    finally:
        ctx.close()


def single_frame_cpp(w, h, reps=50, warm=5):
    """The same single-frame calls as single_frame_timing, driven from C++ (tools/single_frame_c,
    built by __graft_entry__.build()) as the reference's Tracking thread drives them: no Python
    between the calls.  Runs as a child process on the same frames."""
    import tempfile
    from coeb_front import synth
    exe = os.path.join(ROOT, "tools", "single_frame_c")
    if not os.path.exists(exe):
        return dict(skipped="tools/single_frame_c not built (make -C tools)")
    fr = synth.make_frames(w, h, reps + warm + 1, seed=77)
    with tempfile.NamedTemporaryFile(suffix=".u8") as f:
        f.write(fr.tobytes())
        f.flush()
        out = subprocess.run([exe, f.name, str(w), str(h), str(len(fr)), str(warm)], capture_output=True, text=True,
                             timeout=120)
    if out.returncode != 0:
        raise RuntimeError("single_frame_c failed: %s" % out.stderr[-2000:])
    res = json.loads(out.stdout.strip().splitlines()[-1])
    res["note"] = ("median over %d consecutive frames of coeb_extract + coeb_stereo_from_rgbd + coeb_match_lastframe "
                   "(th 15, retry 30), frame i against frame i-1, called from C++ (tools/single_frame_c.cpp)" % reps)
    return res


if __name__ == "__main__":
    main()
