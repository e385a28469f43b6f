#!/bin/bash
# round 5 session 26: k_fm 128 threads (203 VGPRs) and 256 threads at a 3-wave bound (var_fm3: 168
# VGPRs + 32 B scratch) against 256 threads (208 VGPRs) on config D; parity of the 128-thread form
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s26
export TMPDIR=/tmp
COEB_FM_THREADS=128 timeout -k 10 600 python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_parity.py -q -x -m gpu -k "flow or frame_batch or grab_rgbd or fm or moving" --timeout 120 --timeout-method thread > gpurun_out/s26/pt_128.log 2>&1
rc=$?; echo "parity fm=128 rc=$rc $(tail -1 gpurun_out/s26/pt_128.log)"; [ $rc -ne 0 ] && exit $rc
run() {   # tag lib threads
  if [ $2 = main ]; then unset COEB_LIB_PATH; else export COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$2.so; fi
  COEB_FM_THREADS=$3 timeout -k 10 240 python bench.py --config D --steps 20 --warmup 3 --no-cpu-baseline --no-extras --no-e2e > gpurun_out/s26/$1.log 2>&1 || { echo "$1 failed"; tail -5 gpurun_out/s26/$1.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/s26/$1.log') if l.startswith('{')][-1]); k=d['kernels_ms_per_step']; print('%-10s step=%.4f ms value=%.0f k_fm=%.3f' % ('$1', d['ms_per_step'], d['value'], k['k_fm']))"
}
for rep in 1 2; do
  run fm256 main 256
  run fm128 main 128
  run fm256_b3 fm3 256
done
