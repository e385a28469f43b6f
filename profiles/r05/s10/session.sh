#!/bin/bash
# round 5 session 10: speculative buildSystem in k_pose (parity + config D A/B), then configs B
# (shard table) and C on the current build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s10
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -q -x -m gpu -k "pose or track or grab or localmap or flow or frame_batch" --timeout 120 --timeout-method thread > gpurun_out/s10/pt_pose.log 2>&1
rc=$?; echo "pose parity rc=$rc $(tail -1 gpurun_out/s10/pt_pose.log)"; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/s10/pt_pose.log | head; exit $rc; }
KAB_CONFIG=D bash tools/_kab.sh k_pose main lib/var_nospec.so main lib/var_nospec.so || exit 1
cp gpurun_out/kab.log gpurun_out/s10/kabD.log
bash tools/shard_b.sh > gpurun_out/s10/shardB_table.txt 2>&1; rc=$?; cat gpurun_out/s10/shardB_table.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config C --no-cpu-baseline --no-extras > gpurun_out/s10/benchC.log 2>&1 || exit 1
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/s10/benchC.log") if l.startswith("{")][-1])
print("C value", d["value"], "ms/step", d["ms_per_step"], d.get("kernels_ms_per_step"))
PY
