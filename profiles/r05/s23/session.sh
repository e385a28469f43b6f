#!/bin/bash
# round 5 session 23: the whole GPU suite on this build (wave-local pose reduction, shared side
# stream option), then the A / C / D lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s23
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/s23/pytest_gpu.log 2>&1
rc=$?; echo "gpu tests rc=$rc $(tail -1 gpurun_out/s23/pytest_gpu.log)"; [ $rc -ne 0 ] && exit $rc
for c in A C D; do
  timeout -k 10 240 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-extras --no-e2e --no-profile > gpurun_out/s23/$c.log 2>&1 || { echo "$c failed"; tail -5 gpurun_out/s23/$c.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/s23/$c.log') if l.startswith('{')][-1]); print('%s step=%.4f ms value=%.0f side=%s' % ('$c', d['ms_per_step'], d['value'], d['config']['side_stream']))"
done
