#!/bin/bash
# Round 5: config A step time vs hardware-queue count and side stream (the box exports
# GPU_MAX_HW_QUEUES=4).  Each variant one bench run of 40 timed steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/q
echo "box GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}"
one() {
  local tag=$1; shift
  env "$@" timeout -k 10 180 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-extras --no-e2e --no-profile > gpurun_out/q/$tag.log 2>&1 || { echo "$tag rc=$?"; tail -5 gpurun_out/q/$tag.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/q/$tag.log') if l.startswith('{')][-1]); print('%-14s step=%.4f ms value=%.0f' % ('$tag', d['ms_per_step'], d['value']))"
}
for rep in 1 2; do
  one hwq_box
  one side0 COEB_SIDE_STREAM=0
  one hwq8 GPU_MAX_HW_QUEUES=8
  one hwq16 GPU_MAX_HW_QUEUES=16
done
