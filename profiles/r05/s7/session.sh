#!/bin/bash
# round 5 session 7: k_pyr2 (two pyramid levels per launch): pyramid parity, then A/B vs COEB_PYR_FUSE=0
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -m gpu -k "blur_pyramid or golden_extract or extract_A or extract_B or ragged or params or edge_images" --timeout 120 --timeout-method thread > gpurun_out/pt_s7.log 2>&1
rc=$?; echo "parity rc=$rc $(tail -1 gpurun_out/pt_s7.log)"; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/pt_s7.log | head; exit $rc; }
bash tools/_kab.sh k_pyr_level main lib/var_p2rb4.so lib/var_p2rb6.so COEB_PYR_FUSE=0 main
