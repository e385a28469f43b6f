#!/bin/bash
# round 6 session 15: the 64-frame shard with the small-batch octree's doubled LDS key capacity
# (default) vs the plan's (COEB_OCT_KL_SMALL=0, an experiment switch), interleaved repeats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s15; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in default plan; do
    if [ $v = plan ]; then export COEB_EXPERIMENTS=1 COEB_OCT_KL_SMALL=0; else unset COEB_EXPERIMENTS COEB_OCT_KL_SMALL; fi
    timeout -k 10 300 python bench.py --config B --global-frames 64 --steps 60 --warmup 5 --no-cpu-baseline --no-extras --no-e2e > $O/b64_${v}_$rep.log 2>&1 || { tail -3 $O/b64_${v}_$rep.log; exit 1; }
    python -c "import json; d=json.loads([l for l in open('$O/b64_${v}_$rep.log') if l.startswith('{')][-1]); k=d['kernels_ms_per_step']; print('rep $rep $v: %.4f ms/step octree %.4f' % (d['ms_per_step'], k['k_octree']))"
  done
done
