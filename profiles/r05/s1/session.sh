#!/bin/bash
# round 5 session 1: sanity bench, FETCH_SIZE calibration, queue A/B, GPU tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --no-e2e > gpurun_out/b0.log 2>&1
rc=$?; tail -c 400 gpurun_out/b0.log; echo
[ $rc -ne 0 ] && exit $rc
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/calib -o run -- tools/micro/fetch_calib > gpurun_out/calib.log 2>&1
echo "calib rc=$?"
bash tools/r5_queues.sh || exit $?
timeout -k 10 700 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_r5a.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r5a.log; exit $rc
