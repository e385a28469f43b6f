#!/bin/bash
# round 6 session 12: configs[3] shard table on the current build, and the 64-frame shard with
# the matcher's split-list workgroups per pair forced to 2 / 4 / 8 (COEB_MATCH_SPLIT)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s12; mkdir -p $O; export TMPDIR=/tmp
bash tools/shard_b.sh > $O/shard_table.txt 2>&1; cat $O/shard_table.txt
for sp in 2 4 8 0; do
  COEB_MATCH_SPLIT=$sp timeout -k 10 300 python bench.py --config B --global-frames 64 --steps 30 --warmup 3 --no-cpu-baseline --no-extras --no-e2e > $O/b64_split$sp.log 2>&1 || { tail -3 $O/b64_split$sp.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$O/b64_split$sp.log') if l.startswith('{')][-1]); k=d['kernels_ms_per_step']; print('split $sp: %.4f ms/step, match_lists %.4f match %.4f octree %.4f fast %.4f pyr %.4f describe %.4f' % (d['ms_per_step'], k.get('k_match_lists',0), k.get('k_match',0), k.get('k_octree',0), k.get('k_fast',0), k.get('k_pyr_level',0), k.get('k_describe',0)))"
done
