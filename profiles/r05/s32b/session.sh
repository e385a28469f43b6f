#!/bin/bash
# round 5 session 32b: config A, three pipelines of 2048 / 3072 / 4096 frames
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s32b
export TMPDIR=/tmp
run() {   # tag pipelines batch
  timeout -k 10 240 python bench.py --pipelines $2 --batch $3 --steps 12 --warmup 3 --no-cpu-baseline --no-extras --no-e2e --no-profile > gpurun_out/s32b/$1.log 2>&1 || { echo "$1 failed"; tail -5 gpurun_out/s32b/$1.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/s32b/$1.log') if l.startswith('{')][-1]); print('%-10s step=%.4f ms value=%.0f' % ('$1', d['ms_per_step'], d['value']))"
}
for rep in 1 2; do
  run p3x2048 3 6144
  run p3x3072 3 9216
  run p3x4096 3 12288
done
