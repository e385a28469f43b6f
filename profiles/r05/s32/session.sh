#!/bin/bash
# round 5 session 32: config A, pipelines x frames per GPU beyond 3 x 1024
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s32
export TMPDIR=/tmp
run() {   # tag pipelines batch
  timeout -k 10 240 python bench.py --pipelines $2 --batch $3 --steps 20 --warmup 3 --no-cpu-baseline --no-extras --no-e2e --no-profile > gpurun_out/s32/$1.log 2>&1 || { echo "$1 failed"; tail -5 gpurun_out/s32/$1.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/s32/$1.log') if l.startswith('{')][-1]); print('%-10s step=%.4f ms value=%.0f' % ('$1', d['ms_per_step'], d['value']))"
}
for rep in 1 2; do
  run p3x1024 3 3072
  run p3x1365 3 4096
  run p3x1707 3 5120
  run p3x2048 3 6144
  run p2x2048 2 4096
done
