"""bench.parity_check, the checker the bench line's `parity_sample` and the timed-scale GPU tests
(tests/test_gpu_bench_scale.py) use, exercised on the CPU: stand-in pipelines whose per-frame
results come from the oracle run over the WHOLE sequence must be reported bit-exact by the
checker, which recomputes each sampled frame from its own window (frames f-1..f, or f-3..f for the
configs[4] loop: the halo claim of dist.shard_frames, checked here on the oracle itself), and a
single flipped bit in any compared record must be reported."""
import numpy as np
import pytest

import bench
from coeb_front import KEYPOINT_DTYPE, synth


class OraclePipeline:
    """BatchPipeline's frame() surface over results the oracle computed for the whole batch."""

    class _Ctx:
        def __init__(self, stride):
            self.stride = stride

        def batch_results(self):
            return 0, 0, 0, self.stride

    def __init__(self, cfg, F, first=0):
        import oracle as O
        w, h = cfg["w"], cfg["h"]
        self.F = F
        self.ctx = self._Ctx(8 * cfg["nfeatures"] + 256)
        self.recs = []
        if cfg.get("chain"):
            gray, boxes = synth.tracking_sequence(w, h, F, first=first)
            rgb, dep = synth.rgbd_from_gray(gray)
            self.bench_inputs = dict(first=first, rgb=rgb, dep=dep, boxes=boxes)
            cl = bench.ChainCpu(O, cfg, rgb, dep, boxes)
            for f in range(F):
                cl.step(f)
                r, res = cl.last
                rec = dict(kps=r["kps"].copy(), desc=r["desc"].copy())
                if f:
                    rec.update(nmatch=res["nmatches"], match=res["match"].copy(), T1=np.asarray(res["T1"]).copy(),
                               nin1=res["nin1"], T=np.asarray(res["T"]).copy(), ninliers=res["ninliers"],
                               nmatches_map=res["nmatches_map"], nlocal=res["nlocal"],
                               local_match=res["local_match"].copy(), state=res["state"],
                               outlier=res.get("outlier", np.zeros(len(r["kps"]), np.uint8)).copy())
                self.recs.append(rec)
            return
        frames = synth.make_frames(w, h, F, seed=1000, first=first)
        dyn = bench.dyn_batch(w, h, F, first) if cfg.get("dyn") else None
        self.bench_inputs = dict(first=first, frames=frames, dyn=dyn)
        ex = O.Extractor(cfg["nfeatures"], 1.2, 8, 20, 7)
        cam = O.camera(ex, w, h, synth.TUM_FX, synth.TUM_FY, synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
        depth = synth.make_depth(w, h)
        I4 = np.eye(4, dtype=np.float32)
        prev = None
        for f in range(F):
            r = ex.extract(frames[f], *dyn[f]) if dyn else ex.extract(frames[f])
            rec = dict(kps=r["kps"].copy(), desc=r["desc"].copy())
            if prev is not None:
                last = O.mapframe_from_extraction(prev["kps"], prev["desc"], depth, synth.TUM_FX, synth.TUM_FY,
                                                  synth.TUM_CX, synth.TUM_CY, synth.TUM_BF)
                ur, _ = O.stereo_from_rgbd(r["kps"], depth, synth.TUM_BF)
                nm, m = O.search_by_projection(cam, r["kps"], r["desc"], ur, last, synth.motion_pose(), I4, 15.0)
                if nm < 20:
                    nm, m = O.search_by_projection(cam, r["kps"], r["desc"], ur, last, synth.motion_pose(), I4, 30.0)
                rec.update(nmatch=nm, match=m.copy())
            self.recs.append(rec)
            prev = r

    def frame(self, f, track=False):
        return {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in self.recs[f].items()}


@pytest.mark.parametrize("name", ["A", "C"])
def test_parity_check_plain_and_masked(oracle_mod, name):
    cfg = bench.CONFIGS[name]
    bp = OraclePipeline(cfg, 5, first=7)
    r = bench.parity_check([bp], cfg, [[0, 1, 3, 4]])
    assert r["bit_exact"], r["mismatches"]
    assert r["frames"] == 4 and r["matched_frames"] == 3
    rec = bp.recs[3]
    rec["desc"][5, 7] ^= 0x10                               # one descriptor bit
    rec["kps"]["angle"][2] = np.nextafter(rec["kps"]["angle"][2], np.float32(400))   # one angle ulp
    r = bench.parity_check([bp], cfg, [[3]])
    assert not r["bit_exact"]
    assert "angle" in r["mismatches"][0] and "descriptors (1 rows)" in r["mismatches"][0]
    bp.recs[4]["match"][np.argmax(bp.recs[4]["match"] >= 0)] = -1      # one lost match
    r = bench.parity_check([bp], cfg, [[4]])
    assert not r["bit_exact"] and "matches" in r["mismatches"][0]


def test_parity_check_chain_window_equals_whole_sequence(oracle_mod):
    """configs[4]: frame f recomputed from frames f-3..f alone equals frame f of the whole
    sequence, for every frame of an 8-frame run (the 3-frame halo the bench shards with)."""
    cfg = bench.CONFIGS["D"]
    bp = OraclePipeline(cfg, 8)
    assert sum(1 for rc in bp.recs[1:] if rc["state"] == 2) >= 5
    r = bench.parity_check([bp], cfg, [list(range(8))])
    assert r["bit_exact"], r["mismatches"]
    assert r["matched_frames"] == 7
    T = bp.recs[6]["T"]
    T[0, 3] = np.nextafter(T[0, 3], np.float32(1))
    bp.recs[5]["ninliers"] += 1
    r = bench.parity_check([bp], cfg, [[5, 6]])
    assert not r["bit_exact"] and len(r["mismatches"]) == 2
    assert "ninliers" in r["mismatches"][0] and r["mismatches"][1].endswith(": T")


def test_parity_picks():
    p = bench.parity_picks(1025)
    assert {0, 1, 2, 511, 512, 1023, 1024} <= set(p) and len(p) >= 10 and p == sorted(set(p))
    assert bench.parity_picks(3) == [0, 1, 2]
    assert max(bench.parity_picks(257, every=16)) == 256


def test_plan_pipelines_cover_the_sequence():
    for G, world, npipe, halo in ((3072, 1, 3, 1), (512, 1, 2, 1), (3072, 1, 2, 3), (512, 8, 2, 1), (24, 3, 3, 3)):
        seen = []
        for rank in range(world):
            for first, F, nm in bench.plan_pipelines(G, world, rank, npipe, halo):
                assert F - nm >= min(halo, first + F - nm) and first >= 0
                seen += list(range(first + F - nm, first + F))
        assert seen == list(range(1, G + 1))
    assert [s[1] for s in bench.plan_pipelines(3072, 1, 0, 3, 1)] == [1025, 1025, 1025]
    assert KEYPOINT_DTYPE.itemsize == 28
