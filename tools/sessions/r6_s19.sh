#!/bin/bash
# round 6 session 19: k_pyr_rows XCD dealing with magic-number division (main) against round-robin (pyrr0)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s19; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x -m gpu --timeout 120 --timeout-method thread \
    -k "pyramid or golden or extract_A or ragged or params or B_full or batch" > $O/pt.log 2>&1
rc=$?; echo "parity rc=$rc $(tail -1 $O/pt.log)"; [ $rc -ne 0 ] && exit $rc
bash tools/_kab.sh k_pyr_level main lib/var_pyrr0.so main lib/var_pyrr0.so main lib/var_pyrr0.so > $O/kab_pyr.log 2>&1; rc=$?; cat $O/kab_pyr.log; [ $rc -ne 0 ] && exit $rc
KAB_CONFIG=B bash tools/_kab.sh k_pyr_level main lib/var_pyrr0.so main lib/var_pyrr0.so > $O/kab_pyrB.log 2>&1; rc=$?; cat $O/kab_pyrB.log
