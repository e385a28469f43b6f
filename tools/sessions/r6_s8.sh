#!/bin/bash
# round 6 session 8: k_match_local at 512 threads per frame (COEB_LOCAL_NT) -- parity, A/B on D;
# the main build has k_gf_select at 256 threads
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s8; mkdir -p $O; export TMPDIR=/tmp
for v in main loc512; do
  if [ $v = main ]; then unset COEB_LIB_PATH; else export COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$v.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_parity.py -q -x -m gpu --timeout 120 --timeout-method thread \
      -k "localmap or track_local or grab_rgbd or good_features or moving or frame_batch" > $O/pt_$v.log 2>&1
  rc=$?; echo "$v parity rc=$rc $(tail -1 $O/pt_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
unset COEB_LIB_PATH
KAB_CONFIG=D bash tools/_kab.sh k_match_local main lib/var_loc512.so main lib/var_loc512.so > $O/kab_loc.log 2>&1; grep -v "^    " $O/kab_loc.log
