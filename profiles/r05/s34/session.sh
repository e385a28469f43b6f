#!/bin/bash
# round 5 session 34: the k_pose / k_match phase-clock hooks compiled out (build) against compiled in
# (var_clock, the earlier behaviour: a runtime pointer check): config A (k_match) and D (k_pose)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s34
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x -m gpu -k "pose or track or grab_rgbd or match or golden" --timeout 120 --timeout-method thread > gpurun_out/s34/pt.log 2>&1
rc=$?; echo "parity rc=$rc $(tail -1 gpurun_out/s34/pt.log)"; [ $rc -ne 0 ] && exit $rc
run() {   # tag lib config
  if [ $2 = main ]; then unset COEB_LIB_PATH; else export COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$2.so; fi
  timeout -k 10 240 python bench.py --config $3 --steps 10 --warmup 2 --no-cpu-baseline --no-extras --no-e2e > gpurun_out/s34/$1.log 2>&1 || { echo "$1 failed"; tail -5 gpurun_out/s34/$1.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/s34/$1.log') if l.startswith('{')][-1]); k=d['kernels_ms_per_step']; print('%-10s step=%.4f ms value=%.0f k_match=%.4f k_pose=%.4f' % ('$1', d['ms_per_step'], d['value'], k.get('k_match', 0), k.get('k_pose', 0)))"
}
for rep in 1 2; do
  run A_off main A
  run A_on clock A
  run D_off main D
  run D_on clock D
done
