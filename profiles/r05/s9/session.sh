#!/bin/bash
# round 5 session 9: configs B (shard table), C and D on the current build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s9
export TMPDIR=/tmp
bash tools/shard_b.sh > gpurun_out/s9/shardB_table.txt 2>&1; rc=$?; cat gpurun_out/s9/shardB_table.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config C --no-cpu-baseline --no-extras > gpurun_out/s9/benchC.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config D --no-cpu-baseline --no-extras > gpurun_out/s9/benchD.log 2>&1 || exit 1
python - <<'PY'
import json
for t in ("C", "D"):
    d = json.loads([l for l in open("gpurun_out/s9/bench%s.log" % t) if l.startswith("{")][-1])
    print(t, "value", d["value"], "ms/step", d["ms_per_step"], d.get("kernels_ms_per_step"))
PY
