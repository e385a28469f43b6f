#!/bin/bash
# Config B at small shards with 2 / 3 / 4 pipelines: tools/_bpipe.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for g in 64 128 256; do
  for p in 2 3 4 2; do
    timeout -k 10 200 python bench.py --config B --global-frames $g --pipelines $p --no-cpu-baseline --no-extras --no-e2e > gpurun_out/bp.log 2>&1 || { echo "B$g p$p failed"; tail -5 gpurun_out/bp.log; exit 1; }
    python - $g $p <<'PY'
import json, sys
d = json.loads([x for x in open("gpurun_out/bp.log") if x.startswith("{")][-1])
print("B%s pipelines=%s value=%.0f step=%.3f ms" % (sys.argv[1], sys.argv[2], d["value"], d["ms_per_step"]))
PY
  done
done
