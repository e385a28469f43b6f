#!/bin/bash
# round 5 session 3: k_describe variants (IC load batches, LDS-DMA patch staging): parity + A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ddma_icb6 ddma_icb4; do
  COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -m gpu \
     -k "golden_extract or extract_A or extract_B or ragged or params or edge_images or dynamic_masks" --timeout 120 --timeout-method thread > gpurun_out/pt_$v.log 2>&1
  rc=$?; echo "parity $v rc=$rc $(tail -1 gpurun_out/pt_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
bash tools/_kab.sh k_describe main lib/var_icb6.so lib/var_ddma.so lib/var_ddma_icb6.so lib/var_ddma_icb4.so main lib/var_ddma_icb6.so lib/var_ddma_icb4.so
