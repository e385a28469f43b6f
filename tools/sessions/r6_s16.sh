#!/bin/bash
# round 6 session 16: configs[3] shard tables, default and steady-state timed regions
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/s16
bash tools/shard_b.sh > gpurun_out/s16/shardB_table.txt 2>&1; cat gpurun_out/s16/shardB_table.txt
