"""Parity at the timed scale: bench.py's own schedule for each BASELINE config, built by the same
functions rank_main uses (bench.plan_pipelines + bench.make_pipelines: the same pipelines x
frames, the same side-stream mode, the same synthetic input), run for two back-to-back steps with
the pipelines' kernels overlapping exactly as in the timed region, then sampled frames of every
pipeline compared with the oracle bit for bit by bench.parity_check (keypoint records, 256-bit
descriptors, SearchByProjection count and indices with the 2*th retry, and for config D the whole
configs[4] loop's per-frame records).

These launches take the large-batch code paths no smaller test reaches: the 1025-frame octree
plan with its global key spill (F*L > 512), the unsplit 512-thread k_match at P = 1024 pairs
(split lists only below 128 pairs), 1025- and 1537-frame grids, three pipelines with eager or
shared extraction side streams."""
import pytest

import bench

pytestmark = pytest.mark.gpu

# the per-config side-stream environment bench.main() sets before the contexts exist
SIDE_ENV = {"A": {"COEB_SIDE_EAGER": "1", "COEB_SIDE_SHARED": "0"},
            "B": {"COEB_SIDE_EAGER": "0", "COEB_SIDE_SHARED": "0"},
            "C": {"COEB_SIDE_EAGER": "0", "COEB_SIDE_SHARED": "1"},
            "D": {"COEB_SIDE_EAGER": "0", "COEB_SIDE_SHARED": "0"}}


@pytest.mark.parametrize("name", ["A", "C", "B", "D"])
def test_bench_schedule_matches_oracle(monkeypatch, name):
    cfg = bench.CONFIGS[name]
    monkeypatch.delenv("COEB_SIDE_STREAM", raising=False)
    for k, v in SIDE_ENV[name].items():
        monkeypatch.setenv(k, v)
    G = 512 if name == "B" else cfg["batch"]              # B: BASELINE configs[3]'s fixed 512 frames
    halo = 3 if cfg.get("chain") else 1
    subs = bench.plan_pipelines(G, 1, 0, cfg["pipelines"], halo)
    assert len(subs) == cfg["pipelines"] and sum(s[2] for s in subs) == G
    bps = bench.make_pipelines(cfg, subs, 0)
    try:
        kw = bench.step_kwargs(cfg)
        for _ in range(2):
            for bp in bps:                                 # enqueue only, as the timed loop does
                bp.run(**kw)
        for bp in bps:
            bp.synchronize()
        # ~200 frames of A / C (every 16th), ~70 of B (every 8th), ~100 of D (every 32nd): the oracle
        # takes a few seconds for A / B / C, ~20 s for D's four-frame chains
        every = {"A": 16, "C": 16, "B": 8, "D": 32}[name]
        picks = [bench.parity_picks(F, every) for _, F, _ in subs]
        r = bench.parity_check(bps, cfg, picks)
        print(name, {k: r[k] for k in ("frames", "matched_frames", "frames_per_pipeline", "seconds")})
        assert r["frames"] >= 60, r
        assert r["bit_exact"], r["mismatches"]
    finally:
        for bp in bps:
            bp.close()
