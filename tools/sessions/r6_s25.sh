#!/bin/bash
# round 6 session 25: k_subpix slot refill from packed (pair, index) codes (no binary search) -- parity, D A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s25; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_parity.py tests/test_gpu_bench_scale.py -q -x -m gpu --timeout 300 --timeout-method thread \
    -k "flow or subpix or moving or frame_batch or grab or scale" > $O/pt.log 2>&1
rc=$?; echo "parity rc=$rc $(tail -1 $O/pt.log)"; [ $rc -ne 0 ] && exit $rc
KAB_CONFIG=D bash tools/_kab.sh k_subpix main lib/var_fhead.so main lib/var_fhead.so main lib/var_fhead.so > $O/kabD.log 2>&1; rc=$?; grep -v "^    " $O/kabD.log
