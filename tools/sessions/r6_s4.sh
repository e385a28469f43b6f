#!/bin/bash
# round 6 session 4: k_lk derivative taps by buffer loads (COEB_LK_DBUF) -- parity, A/B on config D
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s4; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_flow.py -q -x -m gpu --timeout 120 --timeout-method thread \
    -k "pyramid or golden or extract_A or flow or lk or moving or frame_batch or grab_rgbd" > $O/pt.log 2>&1
rc=$?; echo "parity rc=$rc $(tail -1 $O/pt.log)"; [ $rc -ne 0 ] && exit $rc
KAB_CONFIG=D bash tools/_kab.sh k_lk main lib/var_lkd0.so main lib/var_lkd0.so > $O/kab_lkd.log 2>&1; grep -v "^    " $O/kab_lkd.log
