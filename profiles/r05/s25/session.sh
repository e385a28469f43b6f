#!/bin/bash
# round 5 session 25: k_fm with 256 / 512 / 1024 threads per pair (COEB_FM_THREADS; the 1024-thread
# build spills 208 B per lane at its 128-VGPR bound, 512: 179 VGPRs, 256: 208 VGPRs and two pairs per
# CU): flow parity with each, then config D
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s25
export TMPDIR=/tmp
for t in 256 512; do
  COEB_FM_THREADS=$t timeout -k 10 600 python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_parity.py -q -x -m gpu -k "flow or frame_batch or grab_rgbd or fm or moving" --timeout 120 --timeout-method thread > gpurun_out/s25/pt_$t.log 2>&1
  rc=$?; echo "parity fm=$t rc=$rc $(tail -1 gpurun_out/s25/pt_$t.log)"; [ $rc -ne 0 ] && exit $rc
done
for rep in 1 2; do
  for t in 1024 512 256; do
    COEB_FM_THREADS=$t timeout -k 10 240 python bench.py --config D --steps 20 --warmup 3 --no-cpu-baseline --no-extras --no-e2e > gpurun_out/s25/D_$t.log 2>&1 || { echo "D_$t failed"; tail -5 gpurun_out/s25/D_$t.log; exit 1; }
    python -c "import json; d=json.loads([l for l in open('gpurun_out/s25/D_$t.log') if l.startswith('{')][-1]); k=d['kernels_ms_per_step']; print('D fm=$t step=%.4f ms value=%.0f k_fm=%.3f' % (d['ms_per_step'], d['value'], k['k_fm']))"
  done
done
