#!/bin/bash
# round 5 session 17: describe 16 vs 8 keypoints per wave on configs A, B, C, D (same box)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s17
one() {
  local tag=$1; shift
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras --no-e2e --no-profile "$@" > gpurun_out/s17/$tag.log 2>&1 || { echo "$tag rc=$?"; tail -5 gpurun_out/s17/$tag.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/s17/$tag.log') if l.startswith('{')][-1]); print('%-12s step=%.4f ms value=%.0f' % ('$tag', d['ms_per_step'], d['value']))"
}
K8=$PWD/coeb-slam_amd/lib/var_kp8.so
for rep in 1 2; do
  one A_kp16
  COEB_LIB_PATH=$K8 one A_kp8
  one B_kp16 --config B
  COEB_LIB_PATH=$K8 one B_kp8 --config B
  one C_kp16 --config C
  COEB_LIB_PATH=$K8 one C_kp8 --config C
  one D_kp16 --config D
  COEB_LIB_PATH=$K8 one D_kp8 --config D
done
