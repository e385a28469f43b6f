#!/bin/bash
# Round-4 A/B session 6: config-B 64-frame shard with 1 / 2 / 3 pipelines, side stream on / off.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for pl in 1 2 3; do
  for ss in 1 0; do
    COEB_SIDE_STREAM=$ss timeout -k 10 200 python bench.py --config B --global-frames 64 --pipelines $pl --no-cpu-baseline --no-extras --no-e2e --no-profile > gpurun_out/bp.log 2>&1 || { echo "rc=$?"; tail -3 gpurun_out/bp.log; exit 1; }
    python - $pl $ss <<'PY'
import json, sys
d = json.loads([x for x in open("gpurun_out/bp.log") if x.startswith("{")][-1])
print("B64 pipelines=%s side=%s step=%.3f ms value=%.0f" % (sys.argv[1], sys.argv[2], d["ms_per_step"], d["value"]))
PY
  done
done
