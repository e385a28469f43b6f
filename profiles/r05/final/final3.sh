#!/bin/bash
# round 5 final, part 3: the B and D lines again, now that the committed PMC summaries of B and D carry
# the right frames per launch (their roofline.traffic scales by it)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/final
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --config B > $O/benchB512.log 2>&1 || { tail -5 $O/benchB512.log; exit 1; }
timeout -k 10 600 python bench.py --config D --no-extras > $O/benchD.log 2>&1 || { tail -5 $O/benchD.log; exit 1; }
python - <<'PY'
import json
for t in ("benchB512", "benchD"):
    d = json.loads([l for l in open("gpurun_out/final/%s.log" % t) if l.startswith("{")][-1])
    r = d["roofline"]
    print(t, d["value"], d["ms_per_step"], r.get("kernel"), r.get("frac"), r.get("traffic"), r.get("bytes_per_launch"))
PY
