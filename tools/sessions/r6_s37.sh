#!/bin/bash
# round 6 session 37: k_gf_response Sobel scaling from an LDS table (main) vs HEAD (gfhead) -- parity, D A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s37; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_parity.py tests/test_gpu_bench_scale.py -q -x -m gpu --timeout 300 --timeout-method thread \
    -k "good_features or flow or moving or frame_batch or grab or scale and D" > $O/pt.log 2>&1
rc=$?; echo "parity rc=$rc $(tail -1 $O/pt.log)"; [ $rc -ne 0 ] && exit $rc
KAB_CONFIG=D bash tools/_kab.sh k_gf_response main lib/var_gfhead.so main lib/var_gfhead.so main lib/var_gfhead.so > $O/kabD.log 2>&1; rc=$?; grep -v "^    " $O/kabD.log
