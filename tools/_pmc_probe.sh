#!/bin/bash
# A few PMC passes over a short config-A bench (one pipeline) for k_describe / k_fast diagnosis.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/probe
export TMPDIR=/tmp COEB_SIDE_STREAM=0
B="python bench.py --pipelines 1 --batch 256 --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-e2e --no-extras"
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/probe/p$i -o run -- $B > gpurun_out/probe/p$i.log 2>&1
  rc=$?
  echo "pass $i [$grp] rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 gpurun_out/probe/p$i.log; exit $rc; fi
done
python tools/pmc_summary.py gpurun_out/probe/p*/run_counter_collection.csv > gpurun_out/probe/summary.txt 2>&1
grep -E "^k_" gpurun_out/probe/summary.txt | cut -c1-600
