#!/bin/bash
# round 5 session 43: k_lk takes its points from a queue (build) instead of the fixed grid-stride
# order (var_lkstatic): flow parity, config D
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s43
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_parity.py -q -x -m gpu -k "flow or lk or moving or frame_batch or grab_rgbd" --timeout 120 --timeout-method thread > gpurun_out/s43/pt.log 2>&1
rc=$?; echo "parity rc=$rc $(tail -1 gpurun_out/s43/pt.log)"; [ $rc -ne 0 ] && exit $rc
run() {   # tag lib
  if [ $2 = main ]; then unset COEB_LIB_PATH; else export COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$2.so; fi
  timeout -k 10 240 python bench.py --config D --steps 8 --warmup 2 --no-cpu-baseline --no-extras --no-e2e > gpurun_out/s43/$1.log 2>&1 || { echo "$1 failed"; tail -5 gpurun_out/s43/$1.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/s43/$1.log') if l.startswith('{')][-1]); k=d['kernels_ms_per_step']; print('%-9s step=%.4f ms value=%.0f k_lk=%.4f' % ('$1', d['ms_per_step'], d['value'], k['k_lk']))"
}
for rep in 1 2 3; do
  run queue main
  run static lkstatic
done
