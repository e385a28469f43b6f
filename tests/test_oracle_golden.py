"""The oracle reproduces the committed golden fixtures (tests/golden/make_golden.py)."""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def test_extract_fixture(oracle_mod):
    g = np.load(os.path.join(HERE, "golden", "extract_A.npz"))
    ex = oracle_mod.Extractor()
    for name in ("plain", "dyn", "area"):
        if name == "plain":
            r = ex.extract(g["frame"])
        else:
            r = ex.extract(g["frame"], g[name + "_boxes"], g[name + "_tm"], g[name + "_blur"])
        assert np.array_equal(r["kps"], g[name + "_kps"]), name
        assert np.array_equal(r["desc"], g[name + "_desc"]), name


def test_match_fixture(oracle_mod):
    g = np.load(os.path.join(HERE, "golden", "match_A.npz"))
    ex = oracle_mod.Extractor()
    from coeb_front import synth
    cam = oracle_mod.camera(ex, 640, 480, synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
    last = {k[5:]: g[k] for k in g.files if k.startswith("last_")}
    nm, m = oracle_mod.search_by_projection(cam, g["cur_kps"], g["cur_desc"], g["cur_ur"], last, g["Tcw_cur"],
                                            g["Tcw_last"], 15.0)
    assert nm == int(g["nmatches"]) and np.array_equal(m, g["match"])


def test_synth_deterministic():
    from coeb_front import synth
    a = synth.make_frames(640, 480, 2, seed=1000)
    b = synth.make_frames(640, 480, 2, seed=1000)
    assert np.array_equal(a, b)
    g = np.load(os.path.join(HERE, "golden", "extract_A.npz"))
    assert np.array_equal(a[0], g["frame"])
    # frame 1 is frame 0 translated by (+2, +1) px up to the noise
    d = a[1].astype(int) - np.roll(a[0], (1, 2), axis=(0, 1)).astype(int)
    assert np.abs(d).max() <= 12
