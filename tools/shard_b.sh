#!/bin/bash
# Config B (BASELINE configs[3]: a fixed 512-frame batch at 1280x960, strong scaling) on ONE GPU
# at the per-rank shard sizes of 1 / 2 / 4 / 8 ranks (512 / 256 / 128 / 64 matched frames per
# step).  The predicted strong-scaling efficiency of N ranks is T(512) / (N * T(512 / N)): the
# ranks share no data-path collective, so a rank's step is its shard's time plus the barrier.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/shardB
for g in 512 256 128 64; do
    timeout -k 10 300 python bench.py --config B --global-frames $g --no-cpu-baseline --no-extras \
        > gpurun_out/shardB/g$g.log 2>&1 || { echo "global-frames $g failed rc=$?"; tail -3 gpurun_out/shardB/g$g.log; exit 1; }
done
python - <<'PY'
import json, re
rows = {}
for g in (512, 256, 128, 64):
    line = [l for l in open("gpurun_out/shardB/g%d.log" % g) if l.startswith("{")][-1]
    rows[g] = json.loads(line)
t512 = rows[512]["ms_per_step"]
print("frames/rank  ms/step  frames/s(1 GPU)  predicted N  predicted efficiency")
for g, n in ((512, 1), (256, 2), (128, 4), (64, 8)):
    r = rows[g]
    print("%10d  %7.3f  %15.1f  %11d  %20.3f" % (g, r["ms_per_step"], r["value"], n, t512 / (n * r["ms_per_step"])))
PY
