#!/bin/bash
# round 5 session 41: config D, two pipelines of 1536 / 2048 / 3072 frames
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s41
export TMPDIR=/tmp
run() {   # tag batch
  timeout -k 10 300 python bench.py --config D --batch $2 --steps 8 --warmup 2 --no-cpu-baseline --no-extras --no-e2e --no-profile > gpurun_out/s41/$1.log 2>&1 || { echo "$1 failed"; tail -5 gpurun_out/s41/$1.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/s41/$1.log') if l.startswith('{')][-1]); print('%-8s step=%.4f ms value=%.0f' % ('$1', d['ms_per_step'], d['value']))"
}
for rep in 1 2; do
  run b3072 3072
  run b4096 4096
  run b6144 6144
done
