# PMC passes (one counter group per rocprofv3 run) over a short bench; summary per kernel.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/pmcx
export TMPDIR=/tmp
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-e2e"
i=0
files=""
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmcx/p$i -o run -- $B > gpurun_out/pmcx/p$i.log 2>&1 || { echo "pass $i [$grp] failed rc=$?"; tail -3 gpurun_out/pmcx/p$i.log; exit 1; }
  files="$files gpurun_out/pmcx/p$i/run_counter_collection.csv"
done
python tools/pmc_summary.py $files > gpurun_out/pmcx/summary.txt
grep -E "^k_" gpurun_out/pmcx/summary.txt
