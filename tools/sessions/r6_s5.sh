#!/bin/bash
# round 6 session 5: config D batch / pipelines after the k_lk change
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s5; mkdir -p $O; export TMPDIR=/tmp
for pb in "2 3072" "2 4096" "3 3072" "2 3072" "2 4096" "3 4608"; do
  set -- $pb
  timeout -k 10 300 python bench.py --config D --pipelines $1 --batch $2 --steps 12 --warmup 2 --no-cpu-baseline --no-extras --no-profile > $O/d_$1_$2.log 2>&1 || { echo "fail $pb"; tail -3 $O/d_$1_$2.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$O/d_$1_$2.log') if l.startswith('{')][-1]); print('pipelines %s batch %s: %.0f frames/s, %.3f ms/step' % ('$1', '$2', d['value'], d['ms_per_step']))"
done
