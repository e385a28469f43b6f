#!/bin/bash
# round 5: config A step time vs pipelines per GPU and side stream (box GPU_MAX_HW_QUEUES)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sched
one() {
  local tag=$1; shift
  env "$@" timeout -k 10 180 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extras --no-e2e --no-profile $BARGS > gpurun_out/sched/$tag.log 2>&1 || { echo "$tag rc=$?"; tail -5 gpurun_out/sched/$tag.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/sched/$tag.log') if l.startswith('{')][-1]); print('%-22s step=%.4f ms value=%.0f' % ('$tag', d['ms_per_step'], d['value']))"
}
for rep in 1 2; do
  BARGS="--pipelines 2"; one p2_side
  BARGS="--pipelines 2"; one p2_noside COEB_SIDE_STREAM=0
  BARGS="--pipelines 1"; one p1_side
  BARGS="--pipelines 3 --batch 2049"; one p3_side
  BARGS="--pipelines 3 --batch 2049"; one p3_noside COEB_SIDE_STREAM=0
  BARGS="--pipelines 4"; one p4_noside COEB_SIDE_STREAM=0
  BARGS="--pipelines 2 --batch 4096"; one p2x2048_side
done
