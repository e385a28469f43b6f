#!/bin/bash
# round 6 session 10: config A with k_octree at 128 threads and k_match at 1024 threads per pair
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s10; mkdir -p $O; export TMPDIR=/tmp
for v in oct128 m1024; do
  export COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$v.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -m gpu --timeout 120 --timeout-method thread \
      -k "golden or extract_A or batch_pipeline or split or params" > $O/pt_$v.log 2>&1
  rc=$?; echo "$v parity rc=$rc $(tail -1 $O/pt_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
unset COEB_LIB_PATH
bash tools/_kab.sh k_octree main lib/var_oct128.so lib/var_m1024.so main lib/var_oct128.so lib/var_m1024.so > $O/kab.log 2>&1; grep -v "^    " $O/kab.log
KAB_CONFIG=D bash tools/_kab.sh k_octree main lib/var_oct128.so main lib/var_oct128.so > $O/kabD.log 2>&1; grep -v "^    " $O/kabD.log
