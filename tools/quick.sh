#!/bin/bash
# One quick GPU check of the current tree: the -m gpu suite, then the default bench line (no CPU
# leg, no extras).  Usage: tools/quick.sh TAG [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-q}; shift || true
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/$tag/pytest.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/$tag/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras "$@" > gpurun_out/$tag/bench.log 2>&1
rc=$?
python - "$tag" <<'PY'
import json, sys
t = sys.argv[1]
for l in open("gpurun_out/%s/bench.log" % t):
    if l.startswith("{"):
        d = json.loads(l)
        print("value", d["value"], "ms/step", d["ms_per_step"], "kernels", d.get("kernels_ms_per_step"))
PY
exit $rc
