#!/bin/bash
# round 5 session 40: the flow GPU tests (incl. the k_fm thread-count test) and the sharded tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s40
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_parity.py -v -x -m gpu -k "flow or fm_thread or moving or sharded" --timeout 120 --timeout-method thread > gpurun_out/s40/pt.log 2>&1
rc=$?; echo "rc=$rc $(tail -1 gpurun_out/s40/pt.log)"; grep -c PASSED gpurun_out/s40/pt.log; exit $rc
