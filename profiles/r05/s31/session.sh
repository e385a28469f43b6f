#!/bin/bash
# round 5 session 31: config D's pipelines per GPU after the k_fm change (2 x 512 is the default;
# 3 x 512, 3 x 341, 4 x 256, 2 x 768)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s31
export TMPDIR=/tmp
run() {   # tag pipelines batch
  timeout -k 10 240 python bench.py --config D --pipelines $2 --batch $3 --steps 20 --warmup 3 --no-cpu-baseline --no-extras --no-e2e --no-profile > gpurun_out/s31/$1.log 2>&1 || { echo "$1 failed"; tail -5 gpurun_out/s31/$1.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/s31/$1.log') if l.startswith('{')][-1]); print('%-10s step=%.4f ms value=%.0f' % ('$1', d['ms_per_step'], d['value']))"
}
for rep in 1 2; do  # (round 5 s31b: larger batches below)
  run p2x512 2 1024
  run p3x512 3 1536
  run p3x341 3 1024
  run p4x256 4 1024
  run p2x768 2 1536
done
