#!/bin/bash
# round 5 session 36: configs[3] shard table on the final build, and the 64-frame shard's step
# timeline with the per-kernel alone times of one 33-frame pipeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s36
export TMPDIR=/tmp
bash tools/shard_b.sh > gpurun_out/s36/shardB_table.txt 2>&1 || { cat gpurun_out/s36/shardB_table.txt; exit 1; }
cat gpurun_out/s36/shardB_table.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s36/tl64 -o run -- python bench.py --config B --global-frames 64 --steps 6 --warmup 2 --no-cpu-baseline --no-extras --no-e2e --no-profile > gpurun_out/s36/tl64.log 2>&1 || exit 1
python tools/timeline2.py gpurun_out/s36/tl64/run_kernel_trace.csv 2 > gpurun_out/s36/timeline_b64.txt 2>&1; tail -n 25 gpurun_out/s36/timeline_b64.txt
timeout -k 10 300 python bench.py --config B --global-frames 64 --steps 20 --warmup 3 --no-cpu-baseline --no-extras --no-e2e > gpurun_out/s36/b64.log 2>&1 || exit 1
python -c "import json; d=json.loads([l for l in open('gpurun_out/s36/b64.log') if l.startswith('{')][-1]); print(d['ms_per_step'], d['kernels_ms_per_step'])"
