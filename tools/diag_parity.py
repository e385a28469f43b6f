#!/usr/bin/env python3
"""Stage-by-stage parity diagnostics: HIP path vs the CPU oracle (run on a GPU box).

Prints, per configuration: pyramid byte mismatches per level, FAST candidates per level,
keypoints per level, keypoint-field and descriptor mismatches, matcher agreement.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "coeb-slam_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import oracle as O  # noqa: E402
from coeb_front import Context, synth, make_camera, KEYPOINT_DTYPE  # noqa: E402
import coeb_front  # noqa: E402


def cmp_extract(ctx, ex, gray, boxes=None, tm=None, blur=None, tag=""):
    h, w = gray.shape
    r = ex.extract(gray, boxes, tm, blur, debug=True)
    kps, desc = ctx.extract(gray, boxes, tm, blur)
    sizes = ex.level_sizes(w, h)
    plan_pyr = ctx.debug_read("pyr")
    # pyramid: GPU stores levels 1.. with 256-aligned offsets
    off = 0
    pyr_bad = []
    for l in range(1, len(sizes)):
        lw, lh = sizes[l]
        pitch = (lw + 63) // 64 * 64
        o0 = r["level_off"][l]
        ref = r["pyramid"][o0:o0 + lw * lh].reshape(lh, lw)
        got = plan_pyr[off:off + pitch * lh].reshape(lh, pitch)[:, :lw]
        pyr_bad.append(int((ref != got).sum()))
        off = (off + pitch * lh + 255) // 256 * 256
    lvl_n = ctx.debug_read("lvl_n").view(np.int32)
    print("[%s] area_flag=%d n_ref=%d n_gpu=%d" % (tag, r["area_flag"], len(r["kps"]), len(kps)))
    print("   pyr mismatches per level:", pyr_bad)
    print("   ncand ref:", r["ncand"])
    cn = ctx.debug_read("cand_n").view(np.int32)
    print("   cand_n gpu total:", int(cn.sum()), " ref total:", sum(r["ncand"]))
    print("   nkept ref:", r["nkept"])
    print("   lvl_n gpu:", list(lvl_n))
    ok = len(kps) == len(r["kps"])
    if ok:
        for f in KEYPOINT_DTYPE.names:
            bad = int((kps[f] != r["kps"][f]).sum())
            if bad:
                ok = False
                i = int(np.nonzero(kps[f] != r["kps"][f])[0][0])
                print("   field %s: %d mismatches, first at %d: gpu %r ref %r" % (f, bad, i, kps[i], r["kps"][i]))
        if desc is not None:
            bad = int((desc != r["desc"]).any(axis=1).sum())
            print("   descriptor rows mismatching:", bad)
            ok = ok and bad == 0
    print("   PARITY", "OK" if ok else "FAIL")
    return ok, r, kps, desc


def main():
    ctx = Context(max_width=1280, max_height=960, max_batch=8)
    ex = O.Extractor()
    allok = True
    frames = synth.make_frames(640, 480, 3, seed=1000)
    for i in range(2):
        ok, *_ = cmp_extract(ctx, ex, frames[i], tag="A frame %d" % i)
        allok &= ok
    b, tm, bl = synth.dynamic_inputs(640, 480)
    ok, *_ = cmp_extract(ctx, ex, frames[0], b, tm, bl, tag="A dyn")
    allok &= ok
    b, tm, bl = synth.dynamic_inputs(640, 480, area_flag=True)
    ok, *_ = cmp_extract(ctx, ex, frames[0], b, tm, bl, tag="A dyn area")
    allok &= ok
    fb = synth.make_frames(1280, 960, 1, seed=2000)
    ok, *_ = cmp_extract(ctx, ex, fb[0], tag="B")
    allok &= ok

    # matcher on oracle-extracted frames
    r0 = ex.extract(frames[0])
    r1 = ex.extract(frames[1])
    depth = synth.make_depth(640, 480)
    cam_o = O.camera(ex, 640, 480, synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
    last = O.mapframe_from_extraction(r0["kps"], r0["desc"], depth, synth.TUM_FX, synth.TUM_FY, synth.TUM_CX,
                                      synth.TUM_CY, synth.TUM_BF)
    ur1, _ = O.stereo_from_rgbd(r1["kps"], depth, synth.TUM_BF)
    Tc = synth.motion_pose()
    Tl = np.eye(4, dtype=np.float32)
    nm_ref, m_ref = O.search_by_projection(cam_o, r1["kps"], r1["desc"], ur1, last, Tc, Tl, 15.0)
    cam = make_camera(synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF, 640, 480)
    matcher = coeb_front.ORBmatcher(0.9, True, ctx=ctx)
    cur = coeb_front.Frame(r1["kps"], r1["desc"], ur1, Tcw=Tc)
    lf = coeb_front.Frame(r0["kps"], r0["desc"], Tcw=Tl,
                          map_points=dict(world_pos=last["xw"], descriptor=last["mp_desc"],
                                          observations=last["mp_nobs"], valid=last["has_mp"]))
    nm = matcher.SearchByProjection(cur, lf, 15.0, False, cam)
    mok = nm == nm_ref and np.array_equal(cur.mvpMapPoints, m_ref)
    print("[match] nmatches ref=%d gpu=%d, array equal=%s" % (nm_ref, nm, np.array_equal(cur.mvpMapPoints, m_ref)))
    allok &= mok

    # batch device path vs single-frame path (library-owned device memory; no torch.cuda)
    from coeb_front.pipeline import BatchPipeline
    F = 4
    fr = synth.make_frames(640, 480, F, seed=1000)
    bp = BatchPipeline(640, 480, F)
    bp.load(fr, Tcw=np.stack([synth.motion_pose()] * F))
    bp.run()
    bp.synchronize()
    out, matches, nms = bp.results()
    bok = True
    for f in range(F):
        ref = ex.extract(fr[f])
        kb = out[f][0]
        bok &= len(kb) == len(ref["kps"]) and all(np.array_equal(kb[n], ref["kps"][n]) for n in KEYPOINT_DTYPE.names)
    print("[batch] counts", [len(o[0]) for o in out], "parity", bok, "nmatches", nms[1:])
    allok &= bok
    bp.ctx.profile(True)
    t = time.time()
    for _ in range(5):
        bp.run()
    bp.synchronize()
    print("[time] 5 x batch4: %.3f ms/batch" % ((time.time() - t) / 5 * 1e3))
    print(bp.ctx.profile_read())
    bp.close()
    print("ALL", "OK" if allok else "FAIL")


if __name__ == "__main__":
    main()
