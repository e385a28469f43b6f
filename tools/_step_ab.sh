#!/bin/bash
# Step-time A/B of library variants with long timed loops: tools/_step_ab.sh STEPS lib_a lib_b ...
# ("main" = the in-tree library; each variant runs in turn, the list repeated by the caller)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
n=$1; shift
for v in "$@"; do
  case "$v" in *=*) export "$v"; echo "export $v"; continue;; esac
  if [ "$v" = main ]; then unset COEB_LIB_PATH; else export COEB_LIB_PATH=$PWD/coeb-slam_amd/$v; fi
  timeout -k 10 120 python bench.py --steps $n --warmup 5 --no-cpu-baseline --no-extras --no-e2e --no-profile > gpurun_out/stepab.log 2>&1 || { echo "$v rc=$?"; tail -5 gpurun_out/stepab.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/stepab.log') if l.startswith('{')][-1]); print('%-24s step=%.4f ms value=%.0f' % ('$v', d['ms_per_step'], d['value']))"
done
