#!/bin/bash
# round 5 session 22: k_pose's footprint.  The reduction now stages values per wave (22 KB of LDS
# per frame instead of 62 KB); variants: k_pose<5> at 2 (build) / 3 (var_p5_3) workgroups per CU,
# k_pose<0> (edges read from global memory; COEB_POSE_EPT=0) at 3 (build) / 4 (var_ept0_4)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s22
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -m gpu -k "pose or track or grab_rgbd" --timeout 120 --timeout-method thread > gpurun_out/s22/pt.log 2>&1
rc=$?; echo "parity rc=$rc $(tail -1 gpurun_out/s22/pt.log)"; [ $rc -ne 0 ] && exit $rc
COEB_POSE_EPT=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -m gpu -k "pose or track or grab_rgbd" --timeout 120 --timeout-method thread > gpurun_out/s22/pt0.log 2>&1
rc=$?; echo "parity (k_pose<0>) rc=$rc $(tail -1 gpurun_out/s22/pt0.log)"; [ $rc -ne 0 ] && exit $rc
run() {   # tag lib env...
  local tag=$1 lib=$2; shift 2
  if [ $lib = main ]; then unset COEB_LIB_PATH; else export COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$lib.so; fi
  env "$@" timeout -k 10 240 python bench.py --config D --steps 20 --warmup 3 --no-cpu-baseline --no-extras --no-e2e > gpurun_out/s22/$tag.log 2>&1 || { echo "$tag failed"; tail -5 gpurun_out/s22/$tag.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/s22/$tag.log') if l.startswith('{')][-1]); k=d['kernels_ms_per_step']; print('%-14s step=%.4f ms value=%.0f k_pose=%.3f' % ('$tag', d['ms_per_step'], d['value'], k['k_pose']))"
}
for rep in 1 2; do
  run p5_2_$rep main X=0
  run p5_3_$rep p5_3 X=0
  run p0_3_$rep main COEB_POSE_EPT=0
  run p0_4_$rep ept0_4 COEB_POSE_EPT=0
  run p5_oldred_$rep oldred X=0
done
