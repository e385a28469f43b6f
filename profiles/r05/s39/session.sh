#!/bin/bash
# round 5 session 39: config A (three pipelines, side streams created with their contexts) with 4
# (the box's), 6 and 8 hardware queues per process
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s39
export TMPDIR=/tmp
run() {   # tag queues eager
  GPU_MAX_HW_QUEUES=$2 COEB_SIDE_EAGER=$3 timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras --no-e2e --no-profile > gpurun_out/s39/$1.log 2>&1 || { echo "$1 failed"; tail -5 gpurun_out/s39/$1.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/s39/$1.log') if l.startswith('{')][-1]); print('%-10s step=%.4f ms value=%.0f hwq=%s' % ('$1', d['ms_per_step'], d['value'], d['config']['hw_queues']))"
}
for rep in 1 2 3; do
  run q4e 4 1
  run q6e 6 1
  run q8e 8 1
  run q6l 6 0
done
