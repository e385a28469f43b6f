#!/bin/bash
# round 5 session 29: k_fm<128> with a 2-wave launch bound (build) against the 8-wave bound of
# session 26 (var_fm8; the compiler misses that target and lands on the same 203 VGPRs): config D
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s29
export TMPDIR=/tmp
run() {   # tag lib
  if [ $2 = main ]; then unset COEB_LIB_PATH; else export COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$2.so; fi
  timeout -k 10 240 python bench.py --config D --steps 20 --warmup 3 --no-cpu-baseline --no-extras --no-e2e > gpurun_out/s29/$1.log 2>&1 || { echo "$1 failed"; tail -5 gpurun_out/s29/$1.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/s29/$1.log') if l.startswith('{')][-1]); k=d['kernels_ms_per_step']; print('%-10s step=%.4f ms value=%.0f k_fm=%.3f' % ('$1', d['ms_per_step'], d['value'], k['k_fm']))"
}
for rep in 1 2 3; do
  run b2 main
  run b8 fm8
done
