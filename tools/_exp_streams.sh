#!/bin/bash
# Step time with the batch chunked over 1 / 2 / 3 streams (--streams), two runs each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/streams
for n in 1 2 3 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --streams $n --no-cpu-baseline --no-extras --no-e2e > gpurun_out/streams/s$n.log 2>&1 || { echo "streams $n rc=$?"; tail -5 gpurun_out/streams/s$n.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/streams/s$n.log') if l.startswith('{')][-1]); print('streams $n', d['ms_per_step'], d['value'])"
done
