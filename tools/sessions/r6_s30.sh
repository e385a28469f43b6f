#!/bin/bash
# round 6 session 30: k_subpix 3-row patch ring at a bank-spread slot stride (main) vs the 4-row ring (ring0)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s30; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_parity.py tests/test_gpu_bench_scale.py -q -x -m gpu --timeout 300 --timeout-method thread \
    -k "flow or subpix or moving or frame_batch or grab or scale and D" > $O/pt.log 2>&1
rc=$?; echo "parity rc=$rc $(tail -1 $O/pt.log)"; [ $rc -ne 0 ] && exit $rc
KAB_CONFIG=D bash tools/_kab.sh k_subpix main lib/var_ring0.so main lib/var_ring0.so main lib/var_ring0.so > $O/kabD.log 2>&1; rc=$?; grep -v "^    " $O/kabD.log; [ $rc -ne 0 ] && exit $rc
B="python bench.py --config D --pipelines 2 --batch 1024 --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-e2e --no-extras"
for v in main ring0; do
  if [ $v = main ]; then unset COEB_LIB_PATH; else export COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$v.so; fi
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $O/sq_$v -o run -- $B > $O/sq_$v.log 2>&1 || { echo "pmc $v failed"; exit 1; }
  python - $O/sq_$v/run_counter_collection.csv $v <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    if "k_subpix<" not in r["Kernel_Name"]: continue
    acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
m = {k: sum(v.values()) / max(len(v), 1) for k, v in acc.items()}
print(sys.argv[2], {k: "%.4g" % v for k, v in m.items()}, "conflict/lds_inst %.3f" % (m["SQ_LDS_BANK_CONFLICT"] / max(m["SQ_INSTS_LDS"], 1)))
PY
done
