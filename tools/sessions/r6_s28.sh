#!/bin/bash
# round 6 session 28: candidate index carried in the staged LDS record (one LDS load per candidate) vs HEAD (mhead)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s28; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_scale.py tests/test_gpu_flow.py -q -x -m gpu --timeout 300 --timeout-method thread \
    -k "match or golden or batch or split or retry or kf or local or scale or grab or track or pose" > $O/pt.log 2>&1
rc=$?; echo "parity rc=$rc $(tail -1 $O/pt.log)"; [ $rc -ne 0 ] && exit $rc
COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_mclock.so timeout -k 10 300 python tools/_match_timing.py 640 480 1025 1000 > $O/match_timing_A.txt 2>&1 || { tail -5 $O/match_timing_A.txt; exit 1; }
cat $O/match_timing_A.txt
bash tools/_kab.sh k_match main lib/var_mhead.so main lib/var_mhead.so main lib/var_mhead.so > $O/kab.log 2>&1; rc=$?; grep -v "^    " $O/kab.log; [ $rc -ne 0 ] && exit $rc
KAB_CONFIG=D bash tools/_kab.sh k_match_local main lib/var_mhead.so main lib/var_mhead.so main lib/var_mhead.so > $O/kabD.log 2>&1; rc=$?; cat $O/kabD.log; [ $rc -ne 0 ] && exit $rc
KAB_CONFIG=B bash tools/_kab.sh k_match main lib/var_mhead.so main lib/var_mhead.so > $O/kabB.log 2>&1; grep -v "^    " $O/kabB.log
