#!/bin/bash
# round 6 final, part 1: GPU suite, smoke, the four bench lines with their CPU baselines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_session.sh pytest smoke bench benchB512 benchCfull benchDfull
