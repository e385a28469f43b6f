#!/bin/bash
# round 5 session 33: k_lk launch bound: 1 (build; 99 VGPRs, 4 waves per SIMD), 5 (var_lk5: 94
# VGPRs, 5 waves), 6 (var_lk6: 80 VGPRs + 48 B scratch, 6 waves): flow parity, config D
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s33
export TMPDIR=/tmp
for v in lk5 lk6; do
  COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_flow.py -q -x -m gpu --timeout 120 --timeout-method thread > gpurun_out/s33/pt_$v.log 2>&1
  rc=$?; echo "parity $v rc=$rc $(tail -1 gpurun_out/s33/pt_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
run() {   # tag lib
  if [ $2 = main ]; then unset COEB_LIB_PATH; else export COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$2.so; fi
  timeout -k 10 240 python bench.py --config D --steps 8 --warmup 2 --no-cpu-baseline --no-extras --no-e2e > gpurun_out/s33/$1.log 2>&1 || { echo "$1 failed"; tail -5 gpurun_out/s33/$1.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/s33/$1.log') if l.startswith('{')][-1]); k=d['kernels_ms_per_step']; print('%-8s step=%.4f ms value=%.0f k_lk=%.3f k_subpix=%.3f' % ('$1', d['ms_per_step'], d['value'], k['k_lk'], k['k_subpix']))"
}
for rep in 1 2; do
  run lk1 main
  run lk5 lk5
  run lk6 lk6
done
