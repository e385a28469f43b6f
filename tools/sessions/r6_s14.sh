#!/bin/bash
# round 6 session 14: k_match without the staged current frame (less LDS per pair) on A and D
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s14; mkdir -p $O; export TMPDIR=/tmp
export COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_mnolds.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -m gpu --timeout 120 --timeout-method thread \
    -k "golden or batch_pipeline or split or match or streams" > $O/pt.log 2>&1
rc=$?; echo "mnolds parity rc=$rc $(tail -1 $O/pt.log)"; [ $rc -ne 0 ] && exit $rc
unset COEB_LIB_PATH
bash tools/_kab.sh k_match main lib/var_mnolds.so main lib/var_mnolds.so main lib/var_mnolds.so > $O/kab.log 2>&1; grep -v "^    " $O/kab.log
KAB_CONFIG=D bash tools/_kab.sh k_match main lib/var_mnolds.so main lib/var_mnolds.so > $O/kabD.log 2>&1; grep -v "^    " $O/kabD.log
