#!/bin/bash
# Config B (BASELINE configs[3]: a fixed 512-frame batch at 1280x960, strong scaling) on ONE GPU
# at the per-rank shard sizes of 1 / 2 / 4 / 8 ranks (512 / 256 / 128 / 64 matched frames per
# step).  The predicted strong-scaling efficiency of N ranks is T(512) / (N * T(512 / N)): the
# ranks share no data-path collective, so a rank's step is its shard's time plus the barrier.
# Two tables: the bench's default 20 timed steps per size (a 64-frame shard's timed region is then
# ~14 ms), and steady state with the timed region held at ~90 ms for every size (20 * 512 / g steps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/shardB
for mode in default steady; do
  for g in 512 256 128 64; do
    if [ $mode = steady ]; then st=$(( 20 * 512 / g )); wu=$(( 3 * 512 / g )); else st=20; wu=3; fi
    timeout -k 10 300 python bench.py --config B --global-frames $g --steps $st --warmup $wu --no-cpu-baseline --no-extras \
        --no-e2e > gpurun_out/shardB/${mode}_g$g.log 2>&1 || { echo "global-frames $g failed rc=$?"; tail -3 gpurun_out/shardB/${mode}_g$g.log; exit 1; }
  done
done
python - <<'PY'
import json
for mode in ("default", "steady"):
    rows = {}
    for g in (512, 256, 128, 64):
        line = [l for l in open("gpurun_out/shardB/%s_g%d.log" % (mode, g)) if l.startswith("{")][-1]
        rows[g] = json.loads(line)
    t512 = rows[512]["ms_per_step"]
    print("%s (%s)" % (mode, "20 timed steps per size" if mode == "default" else "20 x 512 / g timed steps"))
    print("frames/rank  steps  ms/step  frames/s(1 GPU)  predicted N  predicted efficiency")
    for g, n in ((512, 1), (256, 2), (128, 4), (64, 8)):
        r = rows[g]
        print("%10d  %5d  %7.3f  %15.1f  %11d  %20.3f" % (g, r["steps"], r["ms_per_step"], r["value"], n, t512 / (n * r["ms_per_step"])))
PY
