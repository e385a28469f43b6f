#!/bin/bash
# round 6 session 39: k_match (512 threads) at 3 waves per SIMD (166 VGPRs, no scratch) vs 4 (128, 108 B scratch)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s39; mkdir -p $O; export TMPDIR=/tmp
COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_w3.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_scale.py -q -x -m gpu \
    --timeout 300 --timeout-method thread -k "match" > $O/pt.log 2>&1
rc=$?; echo "parity(w3) rc=$rc $(tail -1 $O/pt.log)"; [ $rc -ne 0 ] && exit $rc
bash tools/_kab.sh k_match main lib/var_w3.so main lib/var_w3.so main lib/var_w3.so > $O/kabA.log 2>&1; rc=$?; grep -v "^    " $O/kabA.log; [ $rc -ne 0 ] && exit $rc
KAB_CONFIG=B bash tools/_kab.sh k_match main lib/var_w3.so main lib/var_w3.so > $O/kabB.log 2>&1; rc=$?; grep -v "^    " $O/kabB.log
