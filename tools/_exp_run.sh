# Experiment driver for gpurun: GPU tests, then bench variants (one line each).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
i=0
for args in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e $args > gpurun_out/exp_$i.log 2>&1 || { echo "bench [$args] failed rc=$?"; tail -5 gpurun_out/exp_$i.log; exit 1; }
  python - "$args" gpurun_out/exp_$i.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print("[%s] value=%.0f ms/step=%.4f kernels=%s" % (sys.argv[1], d["value"], d["ms_per_step"], d["kernels_ms_per_step"]))
PY
done
