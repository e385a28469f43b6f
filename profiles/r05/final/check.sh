#!/bin/bash
# GPU suite + smoke on the current in-tree build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/check
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/check/pytest_gpu.log 2>&1
rc=$?; echo "gpu tests rc=$rc $(tail -1 gpurun_out/check/pytest_gpu.log)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/check/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 gpurun_out/check/smoke.log)"; exit $rc
