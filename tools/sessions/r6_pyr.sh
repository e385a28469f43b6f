#!/bin/bash
# round 6: k_pyr_rows source-row reuse (COEB_PYR_REUSE) -- parity, then A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/pyr; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -m gpu --timeout 120 --timeout-method thread \
    -k "pyramid or golden or extract_A or ragged or params or batch_pipeline or B_full" > $O/pt.log 2>&1
rc=$?; echo "parity rc=$rc $(tail -1 $O/pt.log)"; [ $rc -ne 0 ] && exit $rc
bash tools/_kab.sh k_pyr_level main lib/var_pyr0.so main lib/var_pyr0.so main lib/var_pyr0.so
