#!/bin/bash
# round 6 session 3: k_pyr_rows source-row reuse and k_lk buffer-load windows -- parity, A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s3; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_flow.py -q -x -m gpu --timeout 120 --timeout-method thread \
    -k "pyramid or golden or extract_A or ragged or params or batch_pipeline or B_full or flow or lk or moving or frame_batch or grab_rgbd" > $O/pt.log 2>&1
rc=$?; echo "parity rc=$rc $(tail -1 $O/pt.log)"; [ $rc -ne 0 ] && exit $rc
bash tools/_kab.sh k_pyr_level main lib/var_pyr0.so main lib/var_pyr0.so main lib/var_pyr0.so > $O/kab_pyr.log 2>&1; cat $O/kab_pyr.log
KAB_CONFIG=D bash tools/_kab.sh k_lk main lib/var_lk0.so main lib/var_lk0.so > $O/kab_lk.log 2>&1; cat $O/kab_lk.log
