#!/bin/bash
# round 5 session 13: config A step, describe with 8 vs 16 keypoints per wave (3 pipelines)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s13
one() {
  local tag=$1; shift
  env "$@" timeout -k 10 180 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-extras --no-e2e --no-profile > gpurun_out/s13/$tag.log 2>&1 || { echo "$tag rc=$?"; tail -5 gpurun_out/s13/$tag.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/s13/$tag.log') if l.startswith('{')][-1]); print('%-10s step=%.4f ms value=%.0f' % ('$tag', d['ms_per_step'], d['value']))"
}
for rep in 1 2 3; do
  one kp8
  one kp16 COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_kp16.so
done
