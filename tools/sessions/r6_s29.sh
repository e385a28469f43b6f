#!/bin/bash
# round 6 session 29: experiment -- large batches build their candidate lists in k_match_lists (512 threads,
# one workgroup per pair), k_match keeps the claims (COEB_MATCH_LISTS1=1); LDS / global-frame lists
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s29; mkdir -p $O; export TMPDIR=/tmp
COEB_EXPERIMENTS=1 COEB_MATCH_LISTS1=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_scale.py tests/test_gpu_parity.py -q -x -m gpu --timeout 300 --timeout-method thread \
    -k "scale and (A or B) or batch_pipeline or golden" > $O/pt.log 2>&1
rc=$?; echo "parity rc=$rc $(tail -1 $O/pt.log)"; [ $rc -ne 0 ] && exit $rc
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --config ${CFG:-A} --steps 10 --warmup 2 --no-cpu-baseline --no-extras --no-e2e > $O/$name.log 2>&1 || { echo "$name failed"; tail -3 $O/$name.log; exit 1; }
  python - $O/$name.log $name <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][0])
k = d["kernels_ms_per_step"]
print("%-10s step=%.4f value=%.0f  lists=%.4f match=%.4f" % (sys.argv[2], d["ms_per_step"], d["value"], k.get("k_match_lists", 0), k.get("k_match", 0)))
PY
}
for r in 1 2 3; do
  run def$r X=1
  run l1_$r COEB_EXPERIMENTS=1 COEB_MATCH_LISTS1=1
  run l1g_$r COEB_EXPERIMENTS=1 COEB_MATCH_LISTS1=1 COEB_MATCH_LISTS_LDS=0
done
