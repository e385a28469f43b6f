#!/bin/bash
# Config D A/B of library variants: tools/_dab.sh lib_a lib_b ... ("main" = the in-tree library;
# ENV=VAL entries are exported for the following runs).  Prints the step and the k_pose time.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "$@"; do
  case "$v" in *=*) export "$v"; echo "export $v"; continue;; esac
  if [ "$v" = main ]; then unset COEB_LIB_PATH; else export COEB_LIB_PATH=$PWD/coeb-slam_amd/$v; fi
  timeout -k 10 240 python bench.py --config D --steps 6 --warmup 2 --no-cpu-baseline --no-extras --no-e2e > gpurun_out/dab.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$v rc=$rc"; tail -5 gpurun_out/dab.log; exit $rc; fi
  python - "$v" <<'PY'
import json, sys
d = json.loads([x for x in open("gpurun_out/dab.log") if x.startswith("{")][0])
k = d["kernels_ms_per_step"]
print("%-24s D value=%.0f step=%.3f ms k_pose=%.3f k_subpix=%.3f k_lk=%.3f k_fm=%.3f" % (sys.argv[1], d["value"],
      d["ms_per_step"], k.get("k_pose", -1), k.get("k_subpix", -1), k.get("k_lk", -1), k.get("k_fm", -1)))
PY
done
