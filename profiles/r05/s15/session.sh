#!/bin/bash
# round 5 session 15: k_describe 16 keypoints per wave with IC loads in batches: kernel alone and step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s15
one() {
  local tag=$1; shift
  env "$@" timeout -k 10 180 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-extras --no-e2e --no-profile > gpurun_out/s15/$tag.log 2>&1 || { echo "$tag rc=$?"; tail -5 gpurun_out/s15/$tag.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/s15/$tag.log') if l.startswith('{')][-1]); print('%-12s step=%.4f ms value=%.0f' % ('$tag', d['ms_per_step'], d['value']))"
}
bash tools/_kab.sh k_describe main lib/var_kp16.so lib/var_kp16b12.so lib/var_kp16b8.so
for rep in 1 2 3; do
  one kp8
  one kp16 COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_kp16.so
  one kp16b12 COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_kp16b12.so
  one kp16b8 COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_kp16b8.so
done
