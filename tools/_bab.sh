#!/bin/bash
# Config B A/B of library variants at one shard size: tools/_bab.sh FRAMES lib_a ENV=VAL main ...
# ("main" = the in-tree library; ENV=VAL entries are exported for the following runs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
g=$1; shift
for v in "$@"; do
  case "$v" in *=*) export "$v"; echo "export $v"; continue;; esac
  if [ "$v" = main ]; then unset COEB_LIB_PATH; else export COEB_LIB_PATH=$PWD/coeb-slam_amd/$v; fi
  timeout -k 10 200 python bench.py --config B --global-frames $g --no-cpu-baseline --no-extras --no-e2e > gpurun_out/bab.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$v rc=$rc"; tail -5 gpurun_out/bab.log; exit $rc; fi
  python - "$v" "$g" <<'PY'
import json, sys
d = json.loads([x for x in open("gpurun_out/bab.log") if x.startswith("{")][-1])
k = d["kernels_ms_per_step"]
print("%-24s B%s value=%.0f step=%.3f ms" % (sys.argv[1], sys.argv[2], d["value"], d["ms_per_step"]))
print("    " + " ".join("%s=%.3f" % (n[2:], v) for n, v in k.items()))
PY
done
