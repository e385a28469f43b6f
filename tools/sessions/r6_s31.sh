#!/bin/bash
# round 6 session 31: k_subpix term rows in two column ranges (half1: 8.8 KB of LDS, 4 waves per SIMD)
# vs one range (main, restructured; shead = the committed build)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s31; mkdir -p $O; export TMPDIR=/tmp
for v in half1 main; do
  if [ $v = main ]; then unset COEB_LIB_PATH; else export COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$v.so; fi
  timeout -k 10 900 python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_parity.py -q -x -m gpu --timeout 300 --timeout-method thread \
      -k "flow or subpix or moving or frame_batch or grab" > $O/pt_$v.log 2>&1
  rc=$?; echo "parity $v rc=$rc $(tail -1 $O/pt_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
unset COEB_LIB_PATH
KAB_CONFIG=D bash tools/_kab.sh k_subpix main lib/var_half1.so lib/var_shead.so main lib/var_half1.so lib/var_shead.so main lib/var_half1.so lib/var_shead.so > $O/kabD.log 2>&1; rc=$?; grep -v "^    " $O/kabD.log
