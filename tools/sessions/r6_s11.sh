#!/bin/bash
# round 6 session 11: cornerSubPix corner slots per wave (6 / 9 / 12) on config D
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s11; mkdir -p $O; export TMPDIR=/tmp
for v in sp6 sp12; do
  export COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$v.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_parity.py -q -x -m gpu --timeout 120 --timeout-method thread \
      -k "subpix or moving or frame_batch or grab_rgbd" > $O/pt_$v.log 2>&1
  rc=$?; echo "$v parity rc=$rc $(tail -1 $O/pt_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
unset COEB_LIB_PATH
KAB_CONFIG=D bash tools/_kab.sh k_subpix main lib/var_sp6.so lib/var_sp12.so main lib/var_sp6.so lib/var_sp12.so > $O/kab.log 2>&1; grep -v "^    " $O/kab.log
