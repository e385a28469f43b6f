#!/bin/bash
# round 5 final evidence on one MI355X: GPU tests, smoke, the bench lines of A (default, with the CPU
# baseline), B, C and D (with the CPU chain baseline), rocprofv3 stats / PMC traffic + VALU passes of
# A, B and D, per-pipe and memory-pipe counters of config A, and the default step's timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/final
mkdir -p $O
export TMPDIR=/tmp
step() {   # name timeout cmd...
    local name=$1 to=$2; shift 2
    local t0=$(date +%s)
    timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc $(( $(date +%s) - t0 ))s"
    if [ $rc -ne 0 ]; then tail -n 5 "$O/$name.log"; exit $rc; fi
}
PART=${1:-all}
if [ "$PART" = all ] || [ "$PART" = 1 ]; then
step pytest_gpu 800 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread
tail -n 2 $O/pytest_gpu.log
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py
step benchB512 600 python bench.py --config B
step benchC 600 python bench.py --config C --no-cpu-baseline --no-extras
step benchD 600 python bench.py --config D --no-extras
python - <<'PY'
import json
for t in ("bench", "benchB512", "benchC", "benchD"):
    d = json.loads([l for l in open("gpurun_out/final/%s.log" % t) if l.startswith("{")][-1])
    cb = d.get("cpu_baseline") or {}
    print(t, "value", d["value"], "ms/step", d["ms_per_step"], "cpu", cb.get("value"), cb.get("spread", {}).get("min"),
          cb.get("spread", {}).get("max"), "roof", d["roofline"].get("kernel"), d["roofline"].get("frac"))
PY
fi
if [ "$PART" = all ] || [ "$PART" = 2 ]; then
bash tools/gpu_session.sh prof profD pmc pmcB pmcD timeline || exit $?
bash tools/pipes.sh final_pipes > $O/pipes.txt 2>&1 || { tail -5 $O/pipes.txt; exit 1; }
bash tools/pipes_mem.sh final_mem > $O/pipes_mem.txt 2>&1 || { tail -5 $O/pipes_mem.txt; exit 1; }
fi
echo done
