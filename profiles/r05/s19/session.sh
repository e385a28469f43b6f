#!/bin/bash
# round 5 session 19: one side stream shared by the device's pipelines (COEB_SIDE_SHARED=1; 3
# context streams + 1 side stream = the 4 hardware queues) vs a side stream per pipeline (default):
# parity under the shared stream, config A and C steps, a kernel timeline of the shared schedule
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s19
export TMPDIR=/tmp
COEB_SIDE_SHARED=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -m gpu -k "golden_extract or extract_A or ragged or dynmask or chunk or split" --timeout 120 --timeout-method thread > gpurun_out/s19/pt.log 2>&1
rc=$?; echo "parity rc=$rc $(tail -1 gpurun_out/s19/pt.log)"; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for v in 0 1; do
    COEB_SIDE_SHARED=$v timeout -k 10 180 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extras --no-e2e --no-profile > gpurun_out/s19/step_$v.log 2>&1 || exit 1
    python -c "import json; d=json.loads([l for l in open('gpurun_out/s19/step_$v.log') if l.startswith('{')][-1]); print('A shared=$v step=%.4f ms value=%.0f' % (d['ms_per_step'], d['value']))"
  done
done
for v in 0 1; do
  COEB_SIDE_SHARED=$v timeout -k 10 180 python bench.py --config C --steps 20 --warmup 5 --no-cpu-baseline --no-extras --no-e2e --no-profile > gpurun_out/s19/stepC_$v.log 2>&1 || exit 1
  python -c "import json; d=json.loads([l for l in open('gpurun_out/s19/stepC_$v.log') if l.startswith('{')][-1]); print('C shared=$v step=%.4f ms value=%.0f' % (d['ms_per_step'], d['value']))"
done
COEB_SIDE_SHARED=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s19/tl -o run -- python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-extras --no-e2e --no-profile > gpurun_out/s19/tl.log 2>&1 || exit 1
python tools/timeline2.py gpurun_out/s19/tl/run_kernel_trace.csv 3 > gpurun_out/s19/timeline.txt 2>&1; tail -n 12 gpurun_out/s19/timeline.txt
# config D's step timeline (which kernels run beside k_pose: it holds 256 VGPRs x 4 waves and
# 62 KB of LDS per frame, two frames per CU)
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s19/tlD -o run -- python bench.py --config D --steps 4 --warmup 2 --no-cpu-baseline --no-extras --no-e2e --no-profile > gpurun_out/s19/tlD.log 2>&1 || exit 1
python tools/timeline2.py gpurun_out/s19/tlD/run_kernel_trace.csv 2 > gpurun_out/s19/timelineD.txt 2>&1; tail -n 30 gpurun_out/s19/timelineD.txt
