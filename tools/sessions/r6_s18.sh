#!/bin/bash
# round 6 session 18: k_pyr_rows workgroup placement -- none (pyrr0) / XCD dealing (main) / frame-major grid (pyrr2)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s18; mkdir -p $O; export TMPDIR=/tmp
COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_pyrr2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x -m gpu --timeout 120 --timeout-method thread \
    -k "pyramid or golden or extract_A or ragged or params or B_full" > $O/pt.log 2>&1
rc=$?; echo "parity pyrr2 rc=$rc $(tail -1 $O/pt.log)"; [ $rc -ne 0 ] && exit $rc
bash tools/_kab.sh k_pyr_level main lib/var_pyrr0.so lib/var_pyrr2.so main lib/var_pyrr0.so lib/var_pyrr2.so main lib/var_pyrr0.so lib/var_pyrr2.so > $O/kab_pyr.log 2>&1; rc=$?; cat $O/kab_pyr.log; [ $rc -ne 0 ] && exit $rc
KAB_CONFIG=B bash tools/_kab.sh k_pyr_level main lib/var_pyrr0.so lib/var_pyrr2.so main lib/var_pyrr0.so lib/var_pyrr2.so > $O/kab_pyrB.log 2>&1; rc=$?; cat $O/kab_pyrB.log; [ $rc -ne 0 ] && exit $rc
export COEB_SIDE_STREAM=0
B="python bench.py --pipelines 1 --batch 1024 --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-e2e --no-extras"
for v in pyrr2; do
  export COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$v.so
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/f_$v -o run -- $B > $O/f_$v.log 2>&1 || { echo "fetch $v failed"; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/w_$v -o run -- $B > $O/w_$v.log 2>&1 || { echo "write $v failed"; exit 1; }
  python tools/pmc_summary.py $O/f_$v/run_counter_collection.csv $O/w_$v/run_counter_collection.csv --json $O/traffic_$v.json --frames 1025 --command "$B" > $O/traffic_$v.log 2>&1
  echo "== $v"; grep pyr $O/traffic_$v.log
done
