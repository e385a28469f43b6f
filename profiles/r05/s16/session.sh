#!/bin/bash
# round 5 session 16: pipelines per GPU for config A with 16-keypoint describe waves
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s16
one() {
  local tag=$1; shift
  timeout -k 10 180 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extras --no-e2e --no-profile "$@" > gpurun_out/s16/$tag.log 2>&1 || { echo "$tag rc=$?"; tail -5 gpurun_out/s16/$tag.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/s16/$tag.log') if l.startswith('{')][-1]); print('%-12s step=%.4f ms value=%.0f' % ('$tag', d['ms_per_step'], d['value']))"
}
for rep in 1 2; do
  one p3x1024 --pipelines 3 --batch 3072
  one p4x1024 --pipelines 4 --batch 4096
  one p2x1024 --pipelines 2 --batch 2048
  one p3x1536 --pipelines 3 --batch 4608
done
