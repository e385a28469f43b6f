#!/bin/bash
# round 5 session 11: pipelines per GPU for config B (512-frame batch and the 64-frame shard) and D
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s11
one() {
  local tag=$1; shift
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras --no-e2e --no-profile "$@" > gpurun_out/s11/$tag.log 2>&1 || { echo "$tag rc=$?"; tail -5 gpurun_out/s11/$tag.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/s11/$tag.log') if l.startswith('{')][-1]); print('%-16s step=%.4f ms value=%.0f' % ('$tag', d['ms_per_step'], d['value']))"
}
for rep in 1 2; do
  one B512_p2 --config B --pipelines 2
  one B512_p3 --config B --pipelines 3
  one B512_p4 --config B --pipelines 4
  one B64_p2 --config B --global-frames 64 --pipelines 2
  one B64_p3 --config B --global-frames 64 --pipelines 3
  one D_p2 --config D --pipelines 2
  one D_p3 --config D --pipelines 3 --batch 1536
done
