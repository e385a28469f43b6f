#!/bin/bash
# round 5 session 6: XCD-aware k_pyr_rows (default) vs round-robin; XCD-aware k_fast variant
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -m gpu -k "blur_pyramid or golden_extract or extract_A or extract_B or ragged or params" --timeout 120 --timeout-method thread > gpurun_out/pt_s6.log 2>&1
rc=$?; echo "parity rc=$rc $(tail -1 gpurun_out/pt_s6.log)"; [ $rc -ne 0 ] && exit $rc
bash tools/_kab.sh k_pyr_level main lib/var_pyrnoremap.so lib/var_fastremap.so main lib/var_pyrnoremap.so lib/var_fastremap.so
