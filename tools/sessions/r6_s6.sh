#!/bin/bash
# round 6 session 6: config D with more hardware queues (3 streams per pipeline: context, side, pose)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s6; mkdir -p $O; export TMPDIR=/tmp
for q in 4 6 8 4 6 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --config D --steps 12 --warmup 2 --no-cpu-baseline --no-extras --no-profile > $O/d_q$q.log 2>&1 || { echo "fail q$q"; tail -3 $O/d_q$q.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$O/d_q$q.log') if l.startswith('{')][-1]); print('hwq %s: %.0f frames/s, %.3f ms/step' % ('$q', d['value'], d['ms_per_step']))"
done
