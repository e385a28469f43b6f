#!/bin/bash
# round 5 session 24: config D with the moving-object batch's LK pyramids (k_pyr_down x4, k_sharr)
# on the side stream beside k_gf_* / k_subpix (default) against all on the context stream
# (COEB_FLOW_SIDE=0)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s24
export TMPDIR=/tmp
COEB_FLOW_SIDE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_parity.py -q -x -m gpu -k "flow or frame_batch or grab_rgbd or pmo or moving" --timeout 120 --timeout-method thread > gpurun_out/s24/pt.log 2>&1
rc=$?; echo "parity rc=$rc $(tail -1 gpurun_out/s24/pt.log)"; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for v in 1 0; do  # 1: fork (opt-in since this session)
    COEB_FLOW_SIDE=$v timeout -k 10 240 python bench.py --config D --steps 20 --warmup 3 --no-cpu-baseline --no-extras --no-e2e --no-profile > gpurun_out/s24/D_$v.log 2>&1 || { echo "D_$v failed"; tail -5 gpurun_out/s24/D_$v.log; exit 1; }
    python -c "import json; d=json.loads([l for l in open('gpurun_out/s24/D_$v.log') if l.startswith('{')][-1]); print('D flow_side=$v step=%.4f ms value=%.0f' % (d['ms_per_step'], d['value']))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s24/tlD -o run -- python bench.py --config D --steps 4 --warmup 2 --no-cpu-baseline --no-extras --no-e2e --no-profile > gpurun_out/s24/tlD.log 2>&1 || exit 1
python tools/timeline2.py gpurun_out/s24/tlD/run_kernel_trace.csv 2 > gpurun_out/s24/timelineD.txt 2>&1; grep "^step" gpurun_out/s24/timelineD.txt
