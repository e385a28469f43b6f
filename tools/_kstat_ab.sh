#!/bin/bash
# Kernel-time A/B of library variants under rocprofv3 --stats:
#   tools/_kstat_ab.sh PATTERN "COMMAND" lib_a lib_b ...   ("main" = the in-tree library)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/kstat
export TMPDIR=/tmp
pat=$1; cmd=$2; shift 2
i=0
for v in "$@"; do
  i=$((i + 1))
  if [ "$v" = main ]; then unset COEB_LIB_PATH; else export COEB_LIB_PATH=$PWD/coeb-slam_amd/$v; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kstat/r$i -o run -- $cmd > gpurun_out/kstat/r$i.log 2>&1 || { echo "$v rc=$?"; tail -5 gpurun_out/kstat/r$i.log; exit 1; }
  python - "$v" "$pat" gpurun_out/kstat/r$i/run_kernel_stats.csv <<'PY'
import csv, re, sys
v, pat, f = sys.argv[1:]
for r in csv.DictReader(open(f)):
    if re.search(pat, r['Name']):
        print("%-24s %-40s calls %4s avg %9.1f us" % (v, r['Name'].replace('(anonymous namespace)::', '')[:40], r['Calls'], float(r['AverageNs']) / 1e3))
PY
done
