#!/bin/bash
# round 5 session 31b: config D, two pipelines with larger batches
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s31b
export TMPDIR=/tmp
run() {   # tag pipelines batch
  timeout -k 10 240 python bench.py --config D --pipelines $2 --batch $3 --steps 12 --warmup 3 --no-cpu-baseline --no-extras --no-e2e --no-profile > gpurun_out/s31b/$1.log 2>&1 || { echo "$1 failed"; tail -5 gpurun_out/s31b/$1.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/s31b/$1.log') if l.startswith('{')][-1]); print('%-10s step=%.4f ms value=%.0f' % ('$1', d['ms_per_step'], d['value']))"
}
for rep in 1 2; do
  run p2x768 2 1536
  run p2x1024 2 2048
  run p2x1536 2 3072
done
