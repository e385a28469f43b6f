#!/bin/bash
# round 6 session 13: the 64-frame shard with 8 (default) vs 4 split-list workgroups per pair, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s13; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2 3; do
  for sp in 8 4 2; do
    COEB_MATCH_SPLIT=$sp timeout -k 10 300 python bench.py --config B --global-frames 64 --steps 60 --warmup 5 --no-cpu-baseline --no-extras --no-e2e --no-profile > $O/b64_split${sp}_$rep.log 2>&1 || { tail -3 $O/b64_split${sp}_$rep.log; exit 1; }
    python -c "import json; d=json.loads([l for l in open('$O/b64_split${sp}_$rep.log') if l.startswith('{')][-1]); print('rep $rep split $sp: %.4f ms/step' % d['ms_per_step'])"
  done
done
