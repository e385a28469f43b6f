#!/bin/bash
# round 5 session 21: how much of config D's step is k_pose's footprint?  A sensitivity variant
# (lib/var_pose1r.so: one LM round of four, NOT bit-exact, never shipped) against the build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s21
export TMPDIR=/tmp
for rep in 1 2; do
  for v in main pose1r; do
    if [ $v = main ]; then unset COEB_LIB_PATH; else export COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$v.so; fi
    timeout -k 10 240 python bench.py --config D --steps 20 --warmup 3 --no-cpu-baseline --no-extras --no-e2e > gpurun_out/s21/D_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/s21/D_$v.log; exit 1; }
    python -c "import json; d=json.loads([l for l in open('gpurun_out/s21/D_$v.log') if l.startswith('{')][-1]); k=d['kernels_ms_per_step']; print('%-8s step=%.4f ms value=%.0f k_pose=%.3f k_fm=%.3f' % ('$v', d['ms_per_step'], d['value'], k['k_pose'], k['k_fm']))"
  done
done
