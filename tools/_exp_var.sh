# Bench ablation variants of the library (coeb-slam_amd/lib/var_<name>.so) without tests.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = base ]; then unset COEB_LIB_PATH; else export COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$v.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --steps 10 > gpurun_out/var_$v.log 2>&1 || { echo "variant $v failed rc=$?"; tail -5 gpurun_out/var_$v.log; exit 1; }
  python - "$v" gpurun_out/var_$v.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print("[%s] value=%.0f ms/step=%.4f kernels=%s" % (sys.argv[1], d["value"], d["ms_per_step"], d["kernels_ms_per_step"]))
PY
done
