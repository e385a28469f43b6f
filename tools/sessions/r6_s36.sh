#!/bin/bash
# round 6 session 36: config A, 2 vs 3 pipelines per GPU (3 interleaved repeats)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s36; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2 3; do
  for pb in "3 3072" "2 3072" "2 4096" "2 2560"; do
    set -- $pb
    timeout -k 10 300 python bench.py --pipelines $1 --batch $2 --steps 20 --warmup 3 --no-cpu-baseline --no-extras --no-e2e --no-profile > $O/p$1_b$2_$r.log 2>&1 || { echo "p$1 b$2 failed"; tail -3 $O/p$1_b$2_$r.log; exit 1; }
    python -c "import json; d=json.loads([l for l in open('$O/p$1_b$2_$r.log') if l.startswith('{')][-1]); print('rep $r pipelines $1 batch $2: %.0f frames/s, %.3f ms/step' % (d['value'], d['ms_per_step']))"
  done
done
