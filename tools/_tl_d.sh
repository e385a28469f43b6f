#!/bin/bash
# Kernel timeline of one config-D step (two pipelines): tools/_tl_d.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tld -o run -- python bench.py --config D --steps 3 --warmup 1 --no-cpu-baseline --no-extras --no-e2e --no-profile > gpurun_out/tld.log 2>&1 || { echo "trace rc=$?"; tail -5 gpurun_out/tld.log; exit 1; }
python tools/timeline2.py gpurun_out/tld/run_kernel_trace.csv 2 > gpurun_out/timeline_d.txt 2>&1; tail -40 gpurun_out/timeline_d.txt
