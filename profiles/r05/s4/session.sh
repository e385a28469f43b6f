#!/bin/bash
# round 5 session 4: tiled blurred pyramid: GPU tests, then A/B against the row-major build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_r5b.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r5b.log; [ $rc -ne 0 ] && exit $rc
bash tools/_kab.sh k_blur main lib/var_rowmajor.so main lib/var_rowmajor.so
