# Bench the default library under environment-variable variants: args "NAME=VAL" or "base".
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = base ]; then envs=""; else envs="$v"; fi
  env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --steps 10 > gpurun_out/env.log 2>&1 || { echo "variant $v failed rc=$?"; tail -5 gpurun_out/env.log; exit 1; }
  python - "$v" gpurun_out/env.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print("[%s] value=%.0f ms/step=%.4f kernels=%s" % (sys.argv[1], d["value"], d["ms_per_step"], d["kernels_ms_per_step"]))
PY
done
