#!/bin/bash
# round 5 session 30: k_fm<128> launch-bound sweep (waves per SIMD 2 = build, 3, 4, 6, 8): the bound
# moves SGPR spills (74 at 2-4, 17 at 6-8) and VGPR scratch (0 / 60-68 B): config D
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s30
export TMPDIR=/tmp
run() {   # tag lib
  if [ $2 = main ]; then unset COEB_LIB_PATH; else export COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$2.so; fi
  timeout -k 10 240 python bench.py --config D --steps 20 --warmup 3 --no-cpu-baseline --no-extras --no-e2e > gpurun_out/s30/$1.log 2>&1 || { echo "$1 failed"; tail -5 gpurun_out/s30/$1.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/s30/$1.log') if l.startswith('{')][-1]); k=d['kernels_ms_per_step']; print('%-10s step=%.4f ms value=%.0f k_fm=%.3f' % ('$1', d['ms_per_step'], d['value'], k['k_fm']))"
}
for rep in 1 2; do
  run b2 main
  run b3 fm3
  run b4 fm4
  run b6 fm6
  run b8 fm8
done
