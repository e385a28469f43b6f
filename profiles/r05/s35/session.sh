#!/bin/bash
# round 5 session 35: cornerSubPix corner slots per wave (COEB_SP_SLOTS; 9 = build: 13.2 KB LDS,
# 3 waves per SIMD; 6/7/8: 9.3/10.6/11.9 KB, 4 waves; 12: 17.2 KB): flow parity, config D
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s35
export TMPDIR=/tmp
for v in sp6 sp8 sp12; do
  COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_flow.py -q -x -m gpu --timeout 120 --timeout-method thread > gpurun_out/s35/pt_$v.log 2>&1
  rc=$?; echo "parity $v rc=$rc $(tail -1 gpurun_out/s35/pt_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
run() {   # tag lib
  if [ $2 = main ]; then unset COEB_LIB_PATH; else export COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$2.so; fi
  timeout -k 10 240 python bench.py --config D --steps 8 --warmup 2 --no-cpu-baseline --no-extras --no-e2e > gpurun_out/s35/$1.log 2>&1 || { echo "$1 failed"; tail -5 gpurun_out/s35/$1.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/s35/$1.log') if l.startswith('{')][-1]); k=d['kernels_ms_per_step']; print('%-8s step=%.4f ms value=%.0f k_subpix=%.3f' % ('$1', d['ms_per_step'], d['value'], k['k_subpix']))"
}
for rep in 1 2; do
  run sp9 main
  run sp6 sp6
  run sp7 sp7
  run sp8 sp8
  run sp12 sp12
done
