#!/bin/bash
# round 6 session 7: k_gf_select threads per pair (COEB_GF_THREADS) -- flow parity per variant, A/B on D
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s7; mkdir -p $O; export TMPDIR=/tmp
for v in gf256 gf512; do
  export COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$v.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_parity.py -q -x -m gpu --timeout 120 --timeout-method thread \
      -k "good_features or moving or frame_batch or grab_rgbd" > $O/pt_$v.log 2>&1
  rc=$?; echo "$v parity rc=$rc $(tail -1 $O/pt_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
unset COEB_LIB_PATH
KAB_CONFIG=D bash tools/_kab.sh k_gf_select main lib/var_gf256.so lib/var_gf512.so main lib/var_gf256.so lib/var_gf512.so > $O/kab_gf.log 2>&1; grep -v "^    " $O/kab_gf.log
grep "^    " $O/kab_gf.log | sed -n 1,3p | cut -c1-200
