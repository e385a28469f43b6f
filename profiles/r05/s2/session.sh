#!/bin/bash
# round 5 session 2: per-pipe counters of the LDS-DMA k_fast build, k_fast at 8 WGs/CU
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/_kab.sh k_fast main lib/var_minwg8.so main lib/var_minwg8.so || exit $?
bash tools/pipes.sh r5pipes1 || exit $?
