#!/usr/bin/env python3
"""Generate the committed golden fixtures from the CPU oracle (oracle/liborb_oracle.so).

Parity status of these vectors: they pin the oracle restatement (regression) and are what
the HIP path is checked against on the GPU box.  They are NOT outputs of the reference
binary (it needs OpenCV 3.4, absent here) -> "parity unpinned" w.r.t. the original build,
see DESIGN.md s3.  Inputs are stored alongside outputs so the fixtures stand alone.

  extract_A.npz : one 640x480 synthetic frame; outputs for (no boxes), (2 boxes + 60 T_M),
                  (3 large boxes -> area_flag)
  match_A.npz   : frame pair 0 -> 1 (LastFrame snapshot + CurrentFrame) and the expected
                  SearchByProjection result for th = 15
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "coeb-slam_amd"))

import numpy as np  # noqa: E402

import oracle as O  # noqa: E402
from coeb_front import synth  # noqa: E402


def main():
    ex = O.Extractor()
    fr = synth.make_frames(640, 480, 2, seed=1000)
    out = dict(frame=fr[0])
    cases = [("plain", None, None, None),
             ("dyn",) + synth.dynamic_inputs(640, 480),
             ("area",) + synth.dynamic_inputs(640, 480, area_flag=True)]
    for name, b, t, bl in cases:
        r = ex.extract(fr[0], b, t, bl)
        out[name + "_kps"] = r["kps"]
        out[name + "_desc"] = r["desc"]
        if b is not None:
            out[name + "_boxes"], out[name + "_tm"], out[name + "_blur"] = b, t, bl
    np.savez_compressed(os.path.join(HERE, "extract_A.npz"), **out)

    r0 = ex.extract(fr[0])
    r1 = ex.extract(fr[1])
    depth = synth.make_depth(640, 480)
    last = O.mapframe_from_extraction(r0["kps"], r0["desc"], depth, synth.TUM_FX, synth.TUM_FY, synth.TUM_CX,
                                      synth.TUM_CY, synth.TUM_BF)
    ur1, _ = O.stereo_from_rgbd(r1["kps"], depth, synth.TUM_BF)
    cam = O.camera(ex, 640, 480, synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
    Tc, Tl = synth.motion_pose(), np.eye(4, dtype=np.float32)
    nm, m = O.search_by_projection(cam, r1["kps"], r1["desc"], ur1, last, Tc, Tl, 15.0)
    np.savez_compressed(os.path.join(HERE, "match_A.npz"), cur_kps=r1["kps"], cur_desc=r1["desc"], cur_ur=ur1,
                        Tcw_cur=Tc, Tcw_last=Tl, nmatches=np.int32(nm), match=m,
                        **{"last_" + k: v for k, v in last.items()})
    print("wrote fixtures: %d/%d/%d keypoints, %d matches" %
          (len(out["plain_kps"]), len(out["dyn_kps"]), len(out["area_kps"]), nm))


if __name__ == "__main__":
    main()
