#!/bin/bash
# round 6 session 33: Context.extract and SearchByProjection(LastFrame) bindings without zero fills / copies -- GPU tests, smoke, A line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/s33
bash tools/gpu_session.sh pytest smoke bench
cp gpurun_out/pytest_gpu.log gpurun_out/smoke.log gpurun_out/bench.log gpurun_out/s33/
