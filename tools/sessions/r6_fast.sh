#!/bin/bash
# round 6: k_fast pre-test passes split from the entry appends (COEB_FAST_SPLITPASS) -- parity of
# each variant, then A/B per-kernel times (config A, side stream as the bench runs it)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/fast; mkdir -p $O; export TMPDIR=/tmp
for v in main var_fsplit var_fsplit2; do
  if [ $v = main ]; then unset COEB_LIB_PATH; else export COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/$v.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -m gpu --timeout 120 --timeout-method thread \
      -k "golden or extract_A or fast or ragged or params or dynamic or batch_pipeline" > $O/pt_$v.log 2>&1
  rc=$?; echo "$v parity rc=$rc $(tail -1 $O/pt_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
unset COEB_LIB_PATH
bash tools/_kab.sh k_fast main lib/var_fsplit.so lib/var_fsplit2.so main lib/var_fsplit.so lib/var_fsplit2.so
