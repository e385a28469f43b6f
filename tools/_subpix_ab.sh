set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for v in ${VARIANTS:-1}; do
  COEB_SUBPIX_VARIANT=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/v$v -o run -- python tools/subpix_ab.py > gpurun_out/ab/v$v.log 2>&1 || { echo "variant $v failed rc=$?"; tail -5 gpurun_out/ab/v$v.log; exit 1; }
  grep iters_per_corner gpurun_out/ab/v$v.log
  python - <<PY
import csv
rows=list(csv.DictReader(open("gpurun_out/ab/v$v/run_kernel_stats.csv")))
for r in rows:
    if 'subpix' in r['Name']: print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,1))
PY
done
