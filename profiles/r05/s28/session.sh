#!/bin/bash
# round 5 session 28: k_fm at 128 threads per pair by default: the whole GPU suite, config D (x2),
# the D timeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s28
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/s28/pytest_gpu.log 2>&1
rc=$?; echo "gpu tests rc=$rc $(tail -1 gpurun_out/s28/pytest_gpu.log)"; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  timeout -k 10 240 python bench.py --config D --steps 20 --warmup 3 --no-cpu-baseline --no-extras --no-e2e > gpurun_out/s28/D.log 2>&1 || { echo "D failed"; tail -5 gpurun_out/s28/D.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/s28/D.log') if l.startswith('{')][-1]); k=d['kernels_ms_per_step']; print('D step=%.4f ms value=%.0f k_fm=%.3f k_pose=%.3f' % (d['ms_per_step'], d['value'], k['k_fm'], k['k_pose']))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s28/tlD -o run -- python bench.py --config D --steps 4 --warmup 2 --no-cpu-baseline --no-extras --no-e2e --no-profile > gpurun_out/s28/tlD.log 2>&1 || exit 1
python tools/timeline2.py gpurun_out/s28/tlD/run_kernel_trace.csv 2 > gpurun_out/s28/timelineD.txt 2>&1; grep -A40 "^step" gpurun_out/s28/timelineD.txt
