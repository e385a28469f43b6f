#!/bin/bash
# round 6 session 27: k_lk blocks dealt to the XCDs in contiguous runs (lkx) vs round-robin (main) -- parity, D A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s27; mkdir -p $O; export TMPDIR=/tmp
COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_lkx.so timeout -k 10 900 python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_parity.py -q -x -m gpu --timeout 300 --timeout-method thread \
    -k "flow or lk or moving or frame_batch or grab" > $O/pt.log 2>&1
rc=$?; echo "parity rc=$rc $(tail -1 $O/pt.log)"; [ $rc -ne 0 ] && exit $rc
KAB_CONFIG=D bash tools/_kab.sh k_lk main lib/var_lkx.so main lib/var_lkx.so main lib/var_lkx.so > $O/kabD.log 2>&1; rc=$?; grep -v "^    " $O/kabD.log
