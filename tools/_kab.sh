#!/bin/bash
# A/B per-kernel times of library variants: tools/_kab.sh KERNEL lib/var_a.so lib/var_b.so ...
# ("main" = the in-tree libcoeb_front.so; ENV=VAL entries are exported for the following runs)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
k=$1; shift
for v in "$@"; do
  case "$v" in *=*) export "$v"; echo "export $v"; continue;; esac
  if [ "$v" = main ]; then unset COEB_LIB_PATH; else export COEB_LIB_PATH=$PWD/coeb-slam_amd/$v; fi
  timeout -k 10 200 python bench.py --config ${KAB_CONFIG:-A} --steps 10 --warmup 2 --no-cpu-baseline --no-extras --no-e2e > gpurun_out/kab.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$v rc=$rc"; tail -5 gpurun_out/kab.log; exit $rc; fi
  python - "$v" "$k" <<'PY'
import json, sys
l = [x for x in open("gpurun_out/kab.log") if x.startswith("{")]
d = json.loads(l[0])
k = d["kernels_ms_per_step"]
print("%-28s %s=%.4f ms  step=%.4f ms  value=%.0f" % (sys.argv[1], sys.argv[2], k.get(sys.argv[2], -1), d["ms_per_step"], d["value"]))
print("    " + " ".join("%s=%.3f" % (n[2:], v) for n, v in k.items()))
PY
done
