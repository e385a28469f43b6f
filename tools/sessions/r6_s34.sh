#!/bin/bash
# round 6 session 34: lazy Frame fields and a leaner stereo call in the single-frame timing -- GPU tests, smoke, A line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/s34
bash tools/gpu_session.sh pytest smoke bench
cp gpurun_out/pytest_gpu.log gpurun_out/smoke.log gpurun_out/bench.log gpurun_out/s34/
