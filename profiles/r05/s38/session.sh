#!/bin/bash
# round 5 session 38: side streams created with their context (COEB_SIDE_EAGER=1: queues taken in
# (context, side) pairs) against created at the first extraction (default): configs A, C, D
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s38
export TMPDIR=/tmp
run() {   # tag config eager
  COEB_SIDE_EAGER=$3 timeout -k 10 240 python bench.py --config $2 --steps 12 --warmup 3 --no-cpu-baseline --no-extras --no-e2e --no-profile > gpurun_out/s38/$1.log 2>&1 || { echo "$1 failed"; tail -5 gpurun_out/s38/$1.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/s38/$1.log') if l.startswith('{')][-1]); print('%-8s step=%.4f ms value=%.0f' % ('$1', d['ms_per_step'], d['value']))"
}
for rep in 1 2 3; do
  run A_lazy A 0
  run A_eager A 1
done
for rep in 1 2; do
  run C_lazy C 0
  run C_eager C 1
  run D_lazy D 0
  run D_eager D 1
done
